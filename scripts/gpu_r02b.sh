#!/bin/bash
# round-2 GPU session B: exact-oracle + ABI tests, bench (host ABI pipeline), PMC of every workload
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02b
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/r02b/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/r02b/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step gpu_tests 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread
step bench_2_2 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline
for t in ${PMC_TAGS:-2_2 2_2ks mb3 4_4}; do
  step pmc_$t 900 bash scripts/pmc_workload.sh $t
done

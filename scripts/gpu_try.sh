#!/bin/bash
# quick A/B session: parity tests of the touched kernels, then bench lines (args: test files; BENCH_TAGS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${TRY_NAME:-try}
mkdir -p $out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -3 "$out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -n "$TRY_TESTS" ]; then
  step tests 600 python -u -m pytest $TRY_TESTS -x -q --timeout 300 --timeout-method thread
fi
for t in ${BENCH_TAGS:-2_2}; do
  step bench_$t 300 python3 bench.py --params $t --steps 5 --warmup 1 --no-cpu-baseline --no-host-abi
done
for t in ${KT_TAGS:-}; do
  step kt_$t 300 rocprofv3 --kernel-trace --stats -d $out/kt_$t -o run --output-format csv -- \
    python3 bench.py --params $t --steps 5 --warmup 1 --no-cpu-baseline --no-host-abi
done
for t in ${PMC_TAGS:-}; do
  step pmc_$t 600 bash scripts/pmc_workload.sh $t
done

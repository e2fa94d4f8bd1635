#!/bin/bash
# round-2 GPU session A: parity tests, smoke, benches of the changed paths
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02a
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/r02a/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/r02a/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_2_2 400 python bench.py --steps 5 --warmup 1
step bench_2_2ks 400 python bench.py --params 2_2ks --steps 5 --warmup 1 --no-cpu-baseline
step bench_mul32 400 python bench.py --params mul32 --steps 3 --warmup 1 --no-cpu-baseline

#!/bin/bash
# round-2 session I: GPU PBS tests (pinned host buffers) and the host-ABI rates of 2_2 / 2_2ks
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r02i
mkdir -p $out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -2 "$out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pbs_tests 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pbs_gpu.py
step bench_2_2 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
step bench_2_2ks 300 python bench.py --params 2_2ks --steps 3 --warmup 1 --no-cpu-baseline

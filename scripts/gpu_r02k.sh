#!/bin/bash
# round-2 session K: N = 32768 two-lane chunk interleave (TFHE_MI355_LARGE_LANES=2): parity under
# the lanes, then 4_4 benches lanes 1 / 2 at chunk sizes CHUNKS (same box)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r02k
mkdir -p $out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -2 "$out/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="--params 4_4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi"
TFHE_MI355_LARGE_LANES=2 step tests_lanes2 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_large_gpu.py
step bench_l1 300 python bench.py $B
for ch in ${CHUNKS:-128 256}; do
  TFHE_MI355_LARGE_LANES=2 TFHE_MI355_LARGE_CHUNK=$ch step bench_l2_c$ch 300 python bench.py $B
done
step bench_l1b 300 python bench.py $B
grep -Ho '"value": [0-9.]*' $out/bench_*.log | cat

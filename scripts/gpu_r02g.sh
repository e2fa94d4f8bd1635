#!/bin/bash
# round-2 session G: bench lines with the SIMD CPU baseline (2_2 headline, 2_2ks, 4_4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r02g
mkdir -p $out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -1 "$out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for t in ${PARAMS:-2_2 2_2ks 4_4}; do
  st=5; [ "$t" = 4_4 ] && st=2
  step bench_$t 500 python bench.py --params $t --steps $st --warmup 1
done

#!/bin/bash
# 2-rank launch rehearsal at HEAD (gloo, both ranks on the one GPU) for the 2_2 and KS+PBS lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r02o
mkdir -p $out
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -1 "$out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step rehearsal_2ranks 400 env BENCH_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi
step rehearsal_2ranks_ks 400 env BENCH_DIST_BACKEND=gloo python bench.py --params 2_2ks --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi

#!/bin/bash
# round-2 session H: config 3 at its full size (65,536 ciphertexts, one call) with the grouped
# CMUX; two-rank launch rehearsal of bench.py --gpus 2 (gloo, both ranks on the one GPU)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r02h
mkdir -p $out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -1 "$out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step rehearsal_2ranks 400 env BENCH_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi
step bench_4_4_full 600 python -u bench.py --params 4_4 --batch 65536 --steps 1 --warmup 0 --no-cpu-baseline --no-host-abi

#!/bin/bash
# N = 32768 path: parity tests, then 4_4 KS+PBS benches of the current build and of variants
# (VARIANTS="name ..." built by scripts/build_variant.sh into tfhe-rs-odd_amd/build/<name>/)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/large_ab
mkdir -p $out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -3 "$out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step tests 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_large_gpu.py tests/test_exact_pbs_gpu.py -k "large or 4_4"
step bench_head 300 python bench.py --params 4_4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi
for v in $VARIANTS; do
  TFHE_MI355_LIB=tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so step bench_$v 300 python bench.py --params 4_4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi
done
for ch in $CHUNKS; do
  TFHE_MI355_LARGE_CHUNK=$ch step bench_c$ch 300 python bench.py --params 4_4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi
done
if [ -n "$KT" ]; then
  step kt 300 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- python3 bench.py --params 4_4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi
fi
grep -ho '"value": [0-9.]*' $out/bench_*.log /dev/null | cat

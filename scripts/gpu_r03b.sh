#!/bin/bash
# Round-3 session B: split/large parity tests at HEAD, then interleaved A/B of library variants
# (VARIANTS, built by scripts/build_variant.sh) on BENCH_TAGS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${RUN_NAME:-r03b}
mkdir -p $out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -n "$TRY_TESTS" ]; then
  TFHE_MI355_LIB=${TEST_VARIANT:+$PWD/tfhe-rs-odd_amd/build/$TEST_VARIANT/libtfhe_mi355.so} \
    step tests 600 python -u -m pytest $TRY_TESTS -x -q --timeout 300 --timeout-method thread
  tail -1 $out/tests.log
fi
for pass in ${PASSES:-1 2}; do
  for v in ${VARIANTS:-}; do
    for t in ${BENCH_TAGS:-4_4}; do
      TFHE_MI355_LIB=$PWD/tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so step b_${v}_${t}_$pass 300 \
        python3 bench.py --params $t --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-host-abi
      grep -o '"value": [0-9.]*\|"large_group_cmux_kernel": [0-9.]*\|"large_dsub_kernel": [0-9.]*\|"large_pair_sub_kernel[^"]*": [0-9.]*' $out/b_${v}_${t}_$pass.log | tail -2 | tr '\n' ' '; echo
    done
  done
done
for t in ${KT_TAGS:-}; do
  step kt_$t 300 rocprofv3 --kernel-trace --stats -d $out/kt_$t -o run --output-format csv -- \
    python3 bench.py --params $t --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi
done

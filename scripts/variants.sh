#!/bin/bash
# A/B kernel variants on one box: parity tests (subset) + bench for each library variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARIANTS:-var1 var2}; do
  lib=tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so
  echo "== $v"
  kexpr=${TESTK-bit_exact}
  TFHE_MI355_LIB=$PWD/$lib timeout -k 10 300 python -m pytest ${TESTFILES:-tests/test_pbs_gpu.py} -x -q ${kexpr:+-k "$kexpr"} > gpurun_out/t_$v.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_$v.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  for bp in ${BENCH_PARAMS:-2_2}; do
    TFHE_MI355_LIB=$PWD/$lib timeout -k 10 300 python bench.py --params $bp --steps 5 --warmup 1 --no-cpu-baseline --no-host-abi > gpurun_out/b_${v}_$bp.log 2>&1
    rc=$?; echo "bench $bp rc=$rc"; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/b_${v}_$bp.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done

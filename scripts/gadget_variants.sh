#!/bin/bash
# A/B of library variants on the fork's gadget parameter sets (bench --params <set>, PBS only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for v in ${VARIANTS:-g0}; do
  lib=$PWD/tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so
  TFHE_MI355_LIB=$lib timeout -k 10 300 python -m pytest tests/test_gadget_params_gpu.py -x -q > gpurun_out/tg_$v.log 2>&1
  rc=$?; echo "== $v tests rc=$rc $(tail -1 gpurun_out/tg_$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  for p in ${SETS:-manticore simon ascon aes40 tfhelib sha3}; do
    TFHE_MI355_LIB=$lib timeout -k 10 200 python bench.py --params $p --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bg_${v}_$p.log 2>&1 || exit $?
    echo "$v $p $(grep -o '"value": [0-9.]*' gpurun_out/bg_${v}_$p.log)"
  done
done

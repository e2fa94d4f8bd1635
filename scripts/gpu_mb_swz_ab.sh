#!/bin/bash
# multi-bit twist-table swizzle A/B: default build vs build/swz5 (round-3 swizzle), mb3 and mb2, two passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for pass in 1 2; do
  for v in base swz5; do
    lib=tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so; [ "$v" = base ] && lib=tfhe-rs-odd_amd/lib/libtfhe_mi355.so
    for p in mb3 mb2; do
      TFHE_MI355_LIB=$lib timeout -k 10 200 python -u bench.py --params $p --steps 5 --warmup 1 --no-cpu-baseline \
        > gpurun_out/r04_mbswz_${v}_${p}_$pass.log 2>&1 || exit 1
    done
  done
done

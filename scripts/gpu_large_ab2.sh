#!/bin/bash
# A/B of large-path variants: bench.py --params $P for each library, two interleaved passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
set -e
for pass in 1 2; do
  for v in ${VARIANTS:-base}; do
    lib=tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so; [ "$v" = base ] && lib=tfhe-rs-odd_amd/lib/libtfhe_mi355.so
    TFHE_MI355_LIB=$lib timeout -k 10 300 python bench.py --params ${P:-3_3} --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-other-workloads > gpurun_out/lab_${P:-3_3}_${v}_$pass.log 2>&1
    grep -o '"value": [0-9.]*' gpurun_out/lab_${P:-3_3}_${v}_$pass.log | head -1
  done
done

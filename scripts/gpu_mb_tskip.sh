#!/bin/bash
# timing-only: multi-bit kernel with conflict-free monomial reads (build/tskipmono) vs default, mb3,
# plus the LDS conflict counters of both (wrong outputs in the variant: the bench's check fails, so
# the rate is read from the log line only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base tskipmono; do
  lib=tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so; [ "$v" = base ] && lib=tfhe-rs-odd_amd/lib/libtfhe_mi355.so
  TFHE_MI355_LIB=$lib timeout -k 10 200 python -u bench.py --params mb3 --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r04_mbtskip_${v}.log 2>&1
  echo "bench $v rc=$?"
  TFHE_MI355_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex pbs_multibit \
    -d gpurun_out/mbtskip_pmc_$v -o run --output-format csv -- python3 bench.py --params mb3 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-host-abi --no-single-call > gpurun_out/mbtskip_pmc_$v.log 2>&1
  echo "pmc $v rc=$?"
done

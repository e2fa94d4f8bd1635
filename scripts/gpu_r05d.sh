#!/bin/bash
# round 5: (1) the multi-bit N = 8192 changes (large_mb_pair2_kernel, large_mb_inv_fwd_kernel): split
# tests + goldens, A/B of the four combinations; (2) the on-chip N = 8192 CMUX (onchip_cmux_kernel):
# split tests + goldens bit-exact, then an A/B against the digits-fed split CMUX at 3_3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py -m gpu -v --timeout 300 --timeout-method thread \
    -k "multi_bit or golden" > gpurun_out/r05_pair2_tests.log 2>&1 || { tail -30 gpurun_out/r05_pair2_tests.log; exit 1; }
tail -3 gpurun_out/r05_pair2_tests.log
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel'), round(d['roofline']['kernel_ms'],4), d['roofline'].get('kernel_times_ms'), d['check'])" "$1"; }
B="--params mb3_3g3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for v in 00 10 01 11; do
  TFHE_MI355_MB_PAIR2=${v:0:1} TFHE_MI355_MB_FUSED=${v:1:1} timeout -k 10 200 python bench.py $B > gpurun_out/r05_ab_mb8_v${v}.json 2> gpurun_out/r05_ab_mb8_v${v}.log || exit 1
  show gpurun_out/r05_ab_mb8_v${v}.json
done
timeout -k 10 900 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py -m gpu -v --timeout 600 --timeout-method thread \
    -k "not multi_bit" > gpurun_out/r05_onchip_tests.log 2>&1 || { tail -30 gpurun_out/r05_onchip_tests.log; exit 1; }
tail -3 gpurun_out/r05_onchip_tests.log
B="--params 3_3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for v in 1 0; do
  TFHE_MI355_ONCHIP=$v timeout -k 10 200 python bench.py $B > gpurun_out/r05_ab_onchip_v${v}.json 2> gpurun_out/r05_ab_onchip_v${v}.log || exit 1
  show gpurun_out/r05_ab_onchip_v${v}.json
done

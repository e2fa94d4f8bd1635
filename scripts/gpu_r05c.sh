#!/bin/bash
# round 5: the multi-bit N = 8192 split CMUX changes -- large_mb_pair2_kernel (monomials from LDS)
# and large_mb_inv_fwd_kernel (top_inv of group i fused with top_fwd of i + 1): split GPU tests and
# goldens bit-exact, then an interleaved same-box A/B of the four combinations (two passes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py -m gpu -v --timeout 300 --timeout-method thread \
    -k "multi_bit or golden" > gpurun_out/r05_pair2_tests.log 2>&1 || { tail -30 gpurun_out/r05_pair2_tests.log; exit 1; }
tail -3 gpurun_out/r05_pair2_tests.log
B="--params mb3_3g3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for pass in 1 2; do
  for v in 00 10 01 11; do
    TFHE_MI355_MB_PAIR2=${v:0:1} TFHE_MI355_MB_FUSED=${v:1:1} timeout -k 10 200 python bench.py $B > gpurun_out/r05_ab_mb8_v${v}_p${pass}.json 2> gpurun_out/r05_ab_mb8_v${v}_p${pass}.log || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel'), round(d['roofline']['kernel_ms'],4), d['roofline'].get('kernel_times_ms'), d['check'])" gpurun_out/r05_ab_mb8_v${v}_p${pass}.json
  done
done
# per-kernel PMC of the shipped configuration (pair2 + fused), for bench.py's roofline entry
export ROUND=r05
timeout -k 10 700 bash scripts/pmc_workload.sh mb3_3g3 > gpurun_out/r05_pmc_mb3_3g3.log 2>&1 || { tail -5 gpurun_out/r05_pmc_mb3_3g3.log; exit 1; }
find gpurun_out/pmc_mb3_3g3 -name '*.csv' -delete
echo pmc ok

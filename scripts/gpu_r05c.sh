#!/bin/bash
# round 5: large_mb_pair2_kernel (multi-bit N = 8192, monomials from LDS): split GPU tests and
# goldens bit-exact, then an interleaved same-box A/B against large_pair_sub_kernel (two passes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py -m gpu -v --timeout 300 --timeout-method thread \
    -k "multi_bit or golden" > gpurun_out/r05_pair2_tests.log 2>&1 || { tail -30 gpurun_out/r05_pair2_tests.log; exit 1; }
tail -3 gpurun_out/r05_pair2_tests.log
B="--params mb3_3g3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for pass in 1 2; do
  for v in 0 1; do
    TFHE_MI355_MB_PAIR2=$v timeout -k 10 200 python bench.py $B > gpurun_out/r05_ab_pair2_v${v}_p${pass}.json 2> gpurun_out/r05_ab_pair2_v${v}_p${pass}.log || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel'), round(d['roofline']['kernel_ms'],4), d['check'])" gpurun_out/r05_ab_pair2_v${v}_p${pass}.json
  done
done

#!/bin/bash
# round 5: the on-chip CMUX for the multi-bit N = 8192 sets -- parity (on-chip vs split vs oracle),
# then an A/B against the split multi-bit path (TFHE_MI355_ONCHIP_MB=0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py -m gpu -v --timeout 600 --timeout-method thread \
    -k "agree or multi_bit or golden" > gpurun_out/r05_onchip_mb_tests.log 2>&1 || { tail -30 gpurun_out/r05_onchip_mb_tests.log; exit 1; }
tail -3 gpurun_out/r05_onchip_mb_tests.log
B="--steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for t in mb3_3g3 mb3_3g2; do
for v in 1 0; do
  TFHE_MI355_ONCHIP_MB=$v timeout -k 10 300 python bench.py --params $t $B > gpurun_out/r05_onchipmb_${t}_v$v.json 2> gpurun_out/r05_onchipmb_${t}_v$v.log || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel_times_ms'), d['check'])" gpurun_out/r05_onchipmb_${t}_v$v.json
done
done

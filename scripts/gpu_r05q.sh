#!/bin/bash
# round 5: the on-chip CMUX at N = 8192, L = 1 (5_1, 6_0) -- parity (on-chip vs split vs oracle), A/B
# against the split path; 3_3 PMC and kernel trace under the kernel's new name (<8192,true,2>)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py -m gpu -v --timeout 600 --timeout-method thread \
    -k "agree or 6_0 or 5_1 or MESSAGE_3_CARRY_3 or golden" > gpurun_out/r05_onchip_l1_tests.log 2>&1 || { tail -30 gpurun_out/r05_onchip_l1_tests.log; exit 1; }
tail -3 gpurun_out/r05_onchip_l1_tests.log
B="--steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for t in 6_0 3_3; do
for v in 1 0; do
  TFHE_MI355_ONCHIP=$v timeout -k 10 300 python bench.py --params $t $B > gpurun_out/r05_onchip_l1_${t}_v$v.json 2> gpurun_out/r05_onchip_l1_${t}_v$v.log || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel'), d['roofline'].get('kernel_times_ms'), d['check'])" gpurun_out/r05_onchip_l1_${t}_v$v.json
done
done
STAGES="kt pmc" KT_TAGS="3_3" PMC_TAGS="3_3" bash scripts/gpu_r05.sh || exit 1

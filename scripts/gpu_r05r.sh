#!/bin/bash
# round 5: the on-chip CMUX at N = 4096 (two ciphertexts per workgroup) -- parity, A/B against the split
# path at 1_4 (L = 2) and 2_3 (L = 1), and a count sweep for the N = 4096 switch
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py -m gpu -v --timeout 600 --timeout-method thread \
    -k "agree or CARRY_4 or CARRY_3 or CARRY_2 or CARRY_1 or CARRY_0 or golden or ragged" > gpurun_out/r05_onchip_4096_tests.log 2>&1 || { tail -30 gpurun_out/r05_onchip_4096_tests.log; exit 1; }
tail -3 gpurun_out/r05_onchip_4096_tests.log
B="--steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for t in 1_4 2_3; do
for v in 1 0; do
  TFHE_MI355_ONCHIP=$v timeout -k 10 300 python bench.py --params $t $B > gpurun_out/r05_onchip_4096_${t}_v$v.json 2> gpurun_out/r05_onchip_4096_${t}_v$v.log || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel'), d['roofline'].get('kernel_times_ms'), d['check'])" gpurun_out/r05_onchip_4096_${t}_v$v.json
done
done
C=1,32,64,96,128,192,256,384,512
for v in 1 0; do
  LAT_PARAMS=PARAM_MESSAGE_1_CARRY_4_KS_PBS TFHE_MI355_ONCHIP=$v TFHE_MI355_ONCHIP_MIN=1 timeout -k 10 400 python scripts/latency_probe.py $C > gpurun_out/r05_sweep14_onchip$v.json 2> gpurun_out/r05_sweep14_onchip$v.log || { tail -5 gpurun_out/r05_sweep14_onchip$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], {k: round(v['ms'],2) for k,v in d['ms'].items()}, all(v['decrypt_ok']==int(k) for k,v in d['ms'].items()))" gpurun_out/r05_sweep14_onchip$v.json
done

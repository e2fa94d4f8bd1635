#!/bin/bash
# round 5: on-chip N = 8192 CMUX -- pair sync after the level L-1 MAC: parity, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py -m gpu -v --timeout 300 --timeout-method thread \
    -k "MESSAGE_3_CARRY_3 or chunks or split_3_3" > gpurun_out/r05_onchip_tests7.log 2>&1 || { tail -30 gpurun_out/r05_onchip_tests7.log; exit 1; }
tail -3 gpurun_out/r05_onchip_tests7.log
B="--params 3_3 --batch 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for pass in 1 2; do
for v in base prev; do
  lib=$PWD/tfhe-rs-odd_amd/lib/libtfhe_mi355.so; [ $v = base ] || lib=$PWD/tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so
  TFHE_MI355_LIB=$lib timeout -k 10 200 python bench.py $B > gpurun_out/r05_ps2_$v.json 2> gpurun_out/r05_ps2_$v.log || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel_times_ms'), d['check'])" gpurun_out/r05_ps2_$v.json
done
done

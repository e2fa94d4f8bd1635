#!/bin/bash
# round 5: N = 4096 on-chip CMUX, one ciphertext per 256-thread workgroup (two per CU) vs two per
# 512-thread workgroup -- parity of the default, A/B at 1_4 and 2_3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py -m gpu -v --timeout 600 --timeout-method thread \
    -k "agree or CARRY_4 or CARRY_3 or CARRY_2 or CARRY_1 or CARRY_0 or golden or ragged" > gpurun_out/r05_onchip_4096b_tests.log 2>&1 || { tail -30 gpurun_out/r05_onchip_4096b_tests.log; exit 1; }
tail -3 gpurun_out/r05_onchip_4096b_tests.log
B="--steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for pass in 1 2; do
for t in 1_4 2_3; do
for v in base cpw2; do
  lib=$PWD/tfhe-rs-odd_amd/lib/libtfhe_mi355.so; [ $v = base ] || lib=$PWD/tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so
  TFHE_MI355_LIB=$lib timeout -k 10 300 python bench.py --params $t $B > gpurun_out/r05_cpw_${t}_$v.json 2> gpurun_out/r05_cpw_${t}_$v.log || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel_times_ms'), d['check'])" gpurun_out/r05_cpw_${t}_$v.json
done
done
done

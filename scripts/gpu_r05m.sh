#!/bin/bash
# round 5: large_mb_pair2_kernel with the GGSW operand batches software pipelined -- parity, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py tests/test_multi_device_gpu.py -m gpu -v --timeout 300 --timeout-method thread \
    -k "multi_bit or golden or multibit" > gpurun_out/r05_mbpipe_tests.log 2>&1 || { tail -30 gpurun_out/r05_mbpipe_tests.log; exit 1; }
tail -3 gpurun_out/r05_mbpipe_tests.log
B="--params mb3_3g3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for pass in 1 2; do
for v in base pipe0; do
  lib=$PWD/tfhe-rs-odd_amd/lib/libtfhe_mi355.so; [ $v = base ] || lib=$PWD/tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so
  TFHE_MI355_LIB=$lib timeout -k 10 200 python bench.py $B > gpurun_out/r05_mbpipe_$v.json 2> gpurun_out/r05_mbpipe_$v.log || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel_times_ms'), d['check'])" gpurun_out/r05_mbpipe_$v.json
done
done

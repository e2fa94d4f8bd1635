#!/bin/bash
# round 5: latency/throughput sweeps for the multi-bit sets (placing kLatPassesMb), then the latency
# and golden tests at the new switch.
set -o pipefail
mkdir -p gpurun_out
C=1,64,128,256,320,512,576,768,896,1024
for g in 3 2; do
  P=PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_${g}_KS_PBS
  LAT_PARAMS=$P TFHE_MI355_LATENCY_MAX=0 timeout -k 10 150 python -u scripts/latency_probe.py $C > gpurun_out/r05_lat_sweep_mb${g}_thr.json 2> gpurun_out/r05_lat_sweep_mb${g}_thr.log || exit 1
  LAT_PARAMS=$P TFHE_MI355_LATENCY_MAX=4096 timeout -k 10 150 python -u scripts/latency_probe.py $C > gpurun_out/r05_lat_sweep_mb${g}_lat.json 2> gpurun_out/r05_lat_sweep_mb${g}_lat.log || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_latency_gpu.py tests/test_golden.py -m gpu -v --timeout 200 --timeout-method thread \
    > gpurun_out/r05_gpu_tests_b.log 2>&1; rc=$?; tail -3 gpurun_out/r05_gpu_tests_b.log; exit $rc

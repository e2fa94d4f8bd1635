#!/bin/bash
# round 5, first GPU pass: the whole -m gpu suite (multi-device contexts included), then the
# latency/throughput kernel sweep over batch sizes 1..1024 at 2_2 (placing the switch).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 720 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread \
    > gpurun_out/r05_gpu_tests_a.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r05_gpu_tests_a.log; exit 1; }
tail -3 gpurun_out/r05_gpu_tests_a.log
C=1,64,128,192,256,320,384,448,512,576,640,704,768,896,1024
TFHE_MI355_LATENCY_MAX=0 timeout -k 10 120 python -u scripts/latency_probe.py $C > gpurun_out/r05_lat_sweep_thr.json 2> gpurun_out/r05_lat_sweep_thr.log &&
TFHE_MI355_LATENCY_MAX=4096 timeout -k 10 120 python -u scripts/latency_probe.py $C > gpurun_out/r05_lat_sweep_lat.json 2> gpurun_out/r05_lat_sweep_lat.log &&
echo sweep ok

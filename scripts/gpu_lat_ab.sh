#!/bin/bash
# latency-kernel variants: device time per batch size (scripts/latency_probe.py), stamps, tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
set -e
run() { local tag=$1 lib=$2 counts=$3; shift 3
  env "$@" TFHE_MI355_LIB=$lib timeout -k 10 240 python scripts/latency_probe.py $counts > gpurun_out/lat_$tag.json 2> gpurun_out/lat_$tag.log; }
B=tfhe-rs-odd_amd/build
run base tfhe-rs-odd_amd/lib/libtfhe_mi355.so 1,64,256,512,1024
run nobf $B/nobf/libtfhe_mi355.so 1,256
run rpw2 $B/rpw2/libtfhe_mi355.so 1,256,512
run st1 $B/stamps/libtfhe_mi355.so 1,256 LAT_STAMPS=1
run st2 $B/stamps2/libtfhe_mi355.so 1,256 LAT_STAMPS=1
timeout -k 10 200 python -u -m pytest tests/test_latency_gpu.py tests/test_golden.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lat_tests.log 2>&1
TFHE_MI355_LIB=$B/rpw2/libtfhe_mi355.so timeout -k 10 200 python -u -m pytest tests/test_latency_gpu.py tests/test_golden.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lat_tests_rpw2.log 2>&1

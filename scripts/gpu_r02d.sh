#!/bin/bash
# round-2 GPU session D: new GPU tests (core_crypto mirror, wire formats), multi-bit lockstep A/B, mb2 PMC
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_core_crypto_gpu.py tests/test_serialization_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02d/tests.log 2>&1
rc=$?; tail -12 gpurun_out/r02d/tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="base mbsync0" TESTFILES="tests/test_multibit_gpu.py" TESTK="" BENCH_PARAMS="mb3 mb2" bash scripts/variants.sh || exit $?
timeout -k 10 600 bash scripts/pmc_workload.sh mb2 > gpurun_out/r02d/pmc_mb2.log 2>&1; rc=$?; tail -3 gpurun_out/r02d/pmc_mb2.log; exit $rc

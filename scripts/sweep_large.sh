#!/bin/bash
# 4_4 bench over chunk sizes (TFHE_MI355_LARGE_CHUNK)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_large_gpu.py > gpurun_out/large_tests.log 2>&1 || { tail -20 gpurun_out/large_tests.log; exit 1; }
tail -1 gpurun_out/large_tests.log
for ch in ${CHUNKS:-64 128 160}; do
  TFHE_MI355_LARGE_CHUNK=$ch timeout -k 10 300 python bench.py --params 4_4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b44_c$ch.log 2>&1 || exit $?
  echo "chunk $ch $(grep -o '"value": [0-9.]*' gpurun_out/b44_c$ch.log)"
done

#!/bin/bash
# bench --params $P under several TFHE_MI355_LARGE_CHUNK values, two interleaved passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
set -e
for pass in 1 2; do
  for c in ${CHUNKS:-256 384 512}; do
    TFHE_MI355_LARGE_CHUNK=$c timeout -k 10 300 python bench.py --params ${P:-3_3} --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call --no-other-workloads > gpurun_out/chunk_${P:-3_3}_${c}_$pass.log 2>&1
    echo "chunk $c pass $pass $(grep -o '"value": [0-9.]*' gpurun_out/chunk_${P:-3_3}_${c}_$pass.log | head -1)"
  done
done

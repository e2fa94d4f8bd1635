#!/bin/bash
# 3_3 (or $P) with the digits-fed CMUX on one lane vs two lanes, two interleaved passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
set -e
for pass in 1 2; do
  for l in 1 2; do
    TFHE_MI355_SPLIT_LANES=$l timeout -k 10 300 python bench.py --params ${P:-3_3} --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-other-workloads > gpurun_out/lanes_${P:-3_3}_${l}_$pass.log 2>&1
    echo "lanes $l pass $pass $(grep -o '"value": [0-9.]*' gpurun_out/lanes_${P:-3_3}_${l}_$pass.log | head -1) $(grep -o '"decrypted_ok": [0-9]*' gpurun_out/lanes_${P:-3_3}_${l}_$pass.log | head -1)"
  done
done

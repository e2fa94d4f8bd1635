#!/bin/bash
# single-call KS+PBS probe under several split-K workgroup targets (TFHE_MI355_KS_SPLIT_WG)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
set -e
for pass in 1 2; do
  for t in ${TARGETS:-256 512 1024 2048}; do
    TFHE_MI355_KS_SPLIT_WG=$t timeout -k 10 200 python scripts/single_call_probe.py 30 > gpurun_out/ksw_${t}_$pass.json 2>/dev/null
    echo "$t $pass $(cat gpurun_out/ksw_${t}_$pass.json)"
  done
done

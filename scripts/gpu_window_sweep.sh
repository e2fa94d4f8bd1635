#!/bin/bash
# coalescer window sweep at 2_2 (TFHE_MI355_COALESCE_WINDOW_US), two passes per setting
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for pass in 1 2; do
  for wu in ${WINDOWS:-500 1000 2000}; do
    TFHE_MI355_COALESCE_WINDOW_US=$wu timeout -k 10 300 python -u bench.py --params 2_2 --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r04_window_${wu}_$pass.log 2>&1 || exit 1
    echo "window $wu pass $pass done"
  done
done

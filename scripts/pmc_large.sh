#!/bin/bash
# Kernel-trace + PMC passes of the N=32768 bench (large_top_fwd / large_sub / large_top_inv),
# one chunk of 128; summarise with scripts/pmc_kernels.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out; export TMPDIR=/tmp
B="python3 bench.py --params 4_4 --batch ${BATCH:-128} --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pl_trace -o run --output-format csv -- $B > gpurun_out/pl_trace.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pl_fetch -o run --output-format csv -- $B > gpurun_out/pl_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pl_write -o run --output-format csv -- $B > gpurun_out/pl_write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAVES -d gpurun_out/pl_sq -o run --output-format csv -- $B > gpurun_out/pl_sq.log 2>&1 || exit $?
echo done

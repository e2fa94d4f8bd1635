#!/bin/bash
# SQ stall-breakdown counters for the 2_2 bench (one rocprofv3 --pmc pass per group).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL"
i=0
P3="SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmc_sq$i -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:---params 2_2 --steps 2 --warmup 1} --no-cpu-baseline > gpurun_out/pmc_sq$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -3 gpurun_out/pmc_sq$i.log
  [ $rc -eq 0 ] || exit $rc
done

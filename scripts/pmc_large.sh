#!/bin/bash
# PMC passes of the N=32768 bench (large_fwd / large_inv kernels).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $grp -d gpurun_out/pmc_large/g$i -o run --output-format csv -- python3 bench.py --params 4_4 --batch 256 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_large_g$i.log 2>&1
  rc=$?; echo "group $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_large_g$i.log; exit $rc; fi
done <<GROUPS
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_WAVES
FETCH_SIZE
WRITE_SIZE
GROUPS

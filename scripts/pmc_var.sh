#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) of bench.py for one library variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out; export TMPDIR=/tmp
v=${VAR:-var3}
export TFHE_MI355_LIB=$PWD/tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so
[ -f "$TFHE_MI355_LIB" ] || export TFHE_MI355_LIB=$PWD/tfhe-rs-odd_amd/lib/libtfhe_mi355.so
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc_$v/g$i -o run --output-format csv -- python3 bench.py --params 2_2 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${v}_g$i.log 2>&1
  rc=$?; echo "group $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${v}_g$i.log; exit $rc; fi
done <<GROUPS
${GROUPS_TXT:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES
FETCH_SIZE
WRITE_SIZE}
GROUPS

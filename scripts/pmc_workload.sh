#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, each under its own time limit) of one bench
# workload, summarised per kernel into gpurun_out/<round>_pmc_<tag>.json (copied to profiles/).
#   usage: pmc_workload.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1
D=gpurun_out/${ROUND:-r04}_pmcraw_$tag
mkdir -p $D
case $tag in
  2_2)   K='pbs_classic_kernel'; U='pbs_classic_kernel'; UPD=4096; M='pbs_classic_kernel'; ARGS="--params 2_2" ;;
  2_2ks) K='pbs_classic_kernel|ks_digits|ks_mfma'; U='pbs_classic_kernel'; UPD=4096; M='pbs_classic_kernel'; ARGS="--params 2_2ks" ;;
  mb3)   K='pbs_multibit'; U='pbs_multibit'; UPD=4096; M='pbs_multibit'; ARGS="--params mb3" ;;
  mb2)   K='pbs_multibit'; U='pbs_multibit'; UPD=4096; M='pbs_multibit'; ARGS="--params mb2" ;;
  4_4)   K='large_|ks_digits|ks_mfma'; U='large_extract_kernel'; UPD=128; M='large_group_cmux_kernel'; ARGS="--params 4_4 --batch 128" ;;
  3_3)   if [ "${TFHE_MI355_ONCHIP:-1}" != 0 ]; then  # the on-chip CMUX: one launch per batch
           K='onchip_|ks_digits|ks_mfma'; U='onchip_cmux_kernel'; UPD=512; M='onchip_cmux_kernel'
         else
           K='large_|split_|ks_digits|ks_mfma'; U='large_extract_kernel'; UPD=512; M='large_dsub_kernel|large_sub_kernel'
         fi; ARGS="--params 3_3 --batch 512" ;;
  1_4|6_0|2_3) K='onchip_|ks_digits|ks_mfma'; U='onchip_cmux_kernel'; UPD=512; M='onchip_cmux_kernel'; ARGS="--params $tag --batch 512" ;;
  mb3_3g2|mb3_3g3) K='large_|split_|ks_digits|ks_mfma'; U='large_extract_kernel'; UPD=1024; M='large_mb_pair2_kernel|large_pair_sub_kernel|large_sub_kernel'; ARGS="--params $tag --batch 1024" ;;
  *) echo "unknown tag $tag"; exit 2 ;;
esac
B="$ARGS ${PMC_EXTRA:-} --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
run() {  # run NAME COUNTERS...
  local n=$1; shift
  # counters only for the workload's own kernels (copy / fill kernels of the runtime excluded)
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d $D/$n -o run --output-format csv -- python3 bench.py $B \
    > $D/$n.log 2>&1
  local rc=$?; echo "pmc $tag $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/$n.log; exit $rc; }
}
if [ "${PMC_TRAFFIC_ONLY:-0}" = 1 ]; then  # L2<->fabric bytes only (the SQ pass crashed under CU-masked lanes)
  run fetch FETCH_SIZE && run write WRITE_SIZE && \
  python3 scripts/pmc_workload.py --fetch $D/fetch --write $D/write --tag $tag --kernels "$K" --unit-kernel "$U" \
    --units-per-dispatch $UPD --main-kernel "$M" --note "${PMC_NOTE:-}" --out gpurun_out/${ROUND:-r04}_pmc_$tag.json
  exit $?
fi
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE && \
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum && \
python3 scripts/pmc_workload.py --fetch $D/fetch --write $D/write \
  --sq $D/sq --extra $D/lds --tag $tag --kernels "$K" --unit-kernel "$U" \
  --units-per-dispatch $UPD --main-kernel "$M" --out gpurun_out/${ROUND:-r04}_pmc_$tag.json

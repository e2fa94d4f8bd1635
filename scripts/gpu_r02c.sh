#!/bin/bash
# round-2 GPU session C: kernel-trace summaries + bench lines of every workload, 4_4 PMC at one chunk
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02c
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/r02c/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/r02c/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for t in ${KT_TAGS:-2_2 2_2ks mb3 mb2 4_4 mul32}; do
  extra="--no-cpu-baseline --no-host-abi"
  [ "$t" = 2_2 ] && extra=""
  st=5; [ "$t" = 4_4 ] && st=2; [ "$t" = mul32 ] && st=3
  step kt_$t 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$t -o run --output-format csv -- \
    python3 bench.py --params $t --steps $st --warmup 1 $extra
done
for t in ${PMC_TAGS:-4_4}; do
  step pmc_$t 900 bash scripts/pmc_workload.sh $t
done

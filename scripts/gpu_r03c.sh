#!/bin/bash
# Round-3 session C: per-kernel PMC summaries (scripts/pmc_workload.sh, one counter group per run)
# and rocprofv3 kernel-trace summaries of the workloads whose kernels changed.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in ${PMC_TAGS:-4_4}; do
  timeout -k 10 600 bash scripts/pmc_workload.sh $t > gpurun_out/pmc_$t.log 2>&1
  rc=$?; echo "== pmc $t rc=$rc"; tail -2 gpurun_out/pmc_$t.log
  [ $rc -eq 0 ] || exit $rc
  find gpurun_out/pmc_$t -name '*.csv' -delete  # raw per-dispatch counters: summarised in r03_pmc_$t.json
done
for t in ${KT_TAGS:-}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$t -o run --output-format csv -- \
    python3 bench.py --params $t --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi > gpurun_out/kt_$t.log 2>&1
  rc=$?; echo "== kt $t rc=$rc"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/kt_$t.log; exit $rc; }
  find gpurun_out/kt_$t -name '*kernel_trace.csv' -delete  # per-dispatch rows; the stats file stays
done

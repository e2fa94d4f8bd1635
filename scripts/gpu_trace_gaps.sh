#!/bin/bash
# Kernel traces of the 3_3 and 4_4 bench workloads at their default batches, summarised by
# scripts/trace_gaps.py (launch gaps between the CMUX kernels) into gpurun_out/r04_trace_gaps_<tag>.txt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SUF=${SUF:-}
for tag in ${TAGS:-3_3 4_4}; do
  d=gpurun_out/trace_$tag$SUF
  timeout -k 10 400 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
    python3 bench.py --params $tag ${EXTRA:---steps 1 --warmup 1} --no-cpu-baseline --no-host-abi --no-single-call \
    > gpurun_out/trace_$tag$SUF.log 2>&1
  rc=$?; echo "trace $tag rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/trace_$tag$SUF.log; exit $rc; }
  f=$(find $d -name '*kernel_trace.csv' | head -n 1)
  python3 scripts/trace_gaps.py "$f" 'large_|split_|ks_' > gpurun_out/r04_trace_gaps_$tag$SUF.txt || exit 1
  grep '^{' gpurun_out/trace_$tag$SUF.log | tail -n 1 | cut -c1-300 >> gpurun_out/r04_trace_gaps_$tag$SUF.txt
  rm -f "$f"
done

#!/bin/bash
# round-2 session L: bench lines (SIMD CPU baseline) + kernel traces of the workloads the classic
# kernel change touches, and the 2_2 PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r02l
mkdir -p $out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -1 "$out/$name.log" | cut -c1-160
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for t in ${PARAMS:-2_2ks mb3 mb2 mul32}; do
  step bench_$t 500 python bench.py --params $t --steps 5 --warmup 1
done
for t in ${KT:-2_2ks mb3 mb2 mul32}; do
  step kt_$t 400 rocprofv3 --kernel-trace --stats -d $out/kt_$t -o run --output-format csv -- \
    python3 bench.py --params $t --steps 5 --warmup 1 --no-cpu-baseline --no-host-abi
done
if [ -n "$PMC" ]; then
  for t in $PMC; do timeout -k 10 900 bash scripts/pmc_workload.sh $t || exit $?; done
fi

#!/bin/bash
# Round-5 GPU session: parity tests, smoke, the default bench (every configuration), rocprofv3
# kernel-trace summaries and per-kernel PMC summaries.  Stages run in order; each GPU step has its
# own time limit and a failing step ends the session (no retries).
#   STAGES="tests smoke bench kt pmc" KT_TAGS="2_2 lat" PMC_TAGS="2_2" bash scripts/gpu_r04.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
for s in ${STAGES:-tests smoke bench}; do
  case $s in
    tests) step r05_gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) step r05_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step r05_bench_default 900 python bench.py --steps 10 --warmup 2 ;;
    rehearse2) step r05_rehearse2_gloo_1gpu 1100 env BENCH_DIST_BACKEND=gloo python -u bench.py --gpus 2 --steps 5 --warmup 1 ;;
    bench22) step r05_bench_2_2 400 python bench.py --params 2_2 --steps 10 --warmup 2 --no-other-workloads ;;
    kt) for t in ${KT_TAGS:-2_2}; do
          if [ "$t" = lat ]; then
            step r05_kt_lat 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_lat -o run --output-format csv -- \
              python3 scripts/latency_probe.py 1,64,256
          elif [ "$t" = latmb3 ]; then
            export LAT_PARAMS=PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS
            step r05_kt_latmb3 300 rocprofv3 --kernel-trace --stats \
              -d gpurun_out/kt_latmb3 -o run --output-format csv -- python3 scripts/latency_probe.py 1,64,256
            unset LAT_PARAMS
          else
            step r05_kt_$t 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$t -o run --output-format csv -- \
              python3 bench.py --params $t --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call --no-other-workloads
          fi
          find gpurun_out/kt_$t -name '*kernel_trace.csv' -delete
        done ;;
    pmc) for t in ${PMC_TAGS:-2_2}; do
           export ROUND=r05
           step r05_pmc_$t 700 bash scripts/pmc_workload.sh $t
           find gpurun_out/pmc_$t -name '*.csv' -delete
         done ;;
  esac
done

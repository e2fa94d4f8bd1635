#!/bin/bash
# Round-6 GPU session: parity tests, smoke, the default bench (every configuration), rocprofv3
# kernel-trace summaries, per-kernel PMC summaries and same-box A/Bs against a variant library.
# Stages run in order; each GPU step has its own time limit and a failing step ends the session
# (no retries).
#   STAGES="tests smoke bench kt pmc" KT_TAGS="2_2 lat" PMC_TAGS="2_2" bash scripts/gpu_r06.sh
#   STAGES="ab" AB_LIB=tfhe-rs-odd_amd/build/old/libtfhe_mi355.so AB_TAGS="3_3 1_4" AB_NAME=launder \
#     bash scripts/gpu_r06.sh
#   STAGES="t" T_FILES="tests/test_split_gpu.py tests/test_golden.py" T_NAME=split bash scripts/gpu_r06.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
# one bench line of workload $1 into gpurun_out/$2.json (stderr $2.log), printed in short
bline() {
  local t=$1 out=$2; shift 2
  timeout -k 10 400 python bench.py --params $t --steps ${AB_STEPS:-5} --warmup 2 --no-cpu-baseline --no-host-abi \
    --no-single-call --no-other-workloads "$@" > gpurun_out/$out.json 2> gpurun_out/$out.log
  local rc=$?; [ $rc -eq 0 ] || { echo "bench $t rc=$rc"; tail -5 gpurun_out/$out.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{}); print(sys.argv[1], round(d['value'],1), r.get('kernel_ms'), r.get('frac'), d.get('check'))" gpurun_out/$out.json
}
for s in ${STAGES:-tests smoke bench}; do
  case $s in
    tests) step r06_gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    t) step r06_tests_${T_NAME:-sel} 600 python -u -m pytest $T_FILES -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) step r06_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step r06_bench_default${BENCH_SUFFIX} 900 python bench.py --steps 10 --warmup 2 ;;
    ctx) step r06_ctx_devices 500 python bench.py --ctx-devices ${CTX_DEVS:-0,0} --steps 3 --warmup 1 ;;
    rehearse2) step r06_rehearse2_gloo_1gpu 1100 env BENCH_DIST_BACKEND=gloo python -u bench.py --gpus 2 --steps 5 --warmup 1 ;;
    ab) for pass in 1 2; do
          for t in ${AB_TAGS:-3_3}; do
            TFHE_MI355_LIB=$AB_LIB bline $t r06_ab_${AB_NAME}_${t}_old$pass ${AB_ARGS}
            bline $t r06_ab_${AB_NAME}_${t}_new$pass ${AB_ARGS}
          done
        done ;;
    probe) # single_call_probe over PROBE_COUNTS at PROBE_PARAMS, once per PROBE_ENVS entry ("name:VAR=x,...")
        for v in ${PROBE_ENVS:-base:X=0}; do
          n=${v%%:*}; e=${v#*:}
          step r06_probe_${PROBE_NAME:-p}_$n 300 env $(echo "$e" | tr ',' ' ') python scripts/single_call_probe.py ${PROBE_REPS:-5} ${PROBE_COUNTS:-1,8,64}
          grep '^{' gpurun_out/r06_probe_${PROBE_NAME:-p}_$n.log
        done ;;
    envab) # ENV_AB="name1:VAR=x,VAR2=y name2:VAR=z" over EAB_TAGS, EAB_PASSES passes, interleaved
        for pass in $(seq 1 ${EAB_PASSES:-2}); do
          for t in ${EAB_TAGS:-4_4}; do
            for v in $ENV_AB; do
              n=${v%%:*}; e=${v#*:}
              env $(echo "$e" | tr ',' ' ') bash -c "$(declare -f bline); bline $t r06_${EAB_NAME:-eab}_${t}_${n}_$pass ${AB_ARGS}" || exit 1
            done
          done
        done ;;
    kt) for t in ${KT_TAGS:-2_2}; do
          if [ "$t" = quad ]; then  # the quad CMUX: single 3_3 KS+PBS calls of 1 and 64 rows
            step ${TAGR:-r06}_kt_quad 300 env PROBE_PARAMS=PARAM_MESSAGE_3_CARRY_3_KS_PBS rocprofv3 --kernel-trace --stats \
              -d gpurun_out/${TAGR:-r06}_kt_quad -o run --output-format csv -- python3 scripts/single_call_probe.py 5 1,64
          elif [ "$t" = lat ]; then
            step ${TAGR:-r06}_kt_lat 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAGR:-r06}_kt_lat -o run --output-format csv -- \
              python3 scripts/latency_probe.py 1,64,256
          else
            step ${TAGR:-r06}_kt_$t 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAGR:-r06}_kt_$t -o run --output-format csv -- \
              python3 bench.py --params $t --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call --no-other-workloads
          fi
          find gpurun_out/${TAGR:-r06}_kt_$t -name '*kernel_trace.csv' -delete
        done ;;
    ktq) # kernel traces of single KS+PBS calls (1 and 64 rows) at each KTQ_PARAMS entry "PARAM_NAME:tag"
        for v in ${KTQ_PARAMS:-PARAM_MESSAGE_3_CARRY_3_KS_PBS:quad}; do
          n=${v#*:}
          step ${TAGR:-r06}_kt_$n 300 env PROBE_PARAMS=${v%%:*} rocprofv3 --kernel-trace --stats \
            -d gpurun_out/${TAGR:-r06}_kt_$n -o run --output-format csv -- python3 scripts/single_call_probe.py 5 1,64
          find gpurun_out/${TAGR:-r06}_kt_$n -name '*kernel_trace.csv' -delete
        done ;;
    pmc) for t in ${PMC_TAGS:-2_2}; do
           export ROUND=${TAGR:-r06}
           step ${TAGR:-r06}_pmc_$t 700 bash scripts/pmc_workload.sh $t
           find gpurun_out/${TAGR:-r06}_pmcraw_$t -name '*.csv' -delete
         done ;;
  esac
done

#!/bin/bash
# One GPU-box session of round 3: GPU parity tests, smoke, the default bench run, per-workload
# rocprofv3 kernel-trace summaries and per-kernel PMC passes.  Each GPU step has its own time
# limit; a crash / abort / timeout (rc not 0 or 1) stops the script.
#   STAGES="tests smoke bench kstats:2_2 pmc:2_2 ..." scripts/gpu_r03.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  # heartbeat: a step that prints nothing for minutes (keygen, rocprofv3 passes) is not hung
  ( while sleep 45; do echo "   $name running $(date +%T)"; done ) & local hb=$!
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; kill $hb 2>/dev/null; wait $hb 2>/dev/null
  echo "== $name rc=$rc $(date +%T)"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
kargs() {  # bench arguments of a kernel-trace / PMC run of one workload
  case $1 in
    4_4) echo "--params 4_4 --batch 1024 --steps 2 --warmup 1" ;;
    3_3|mb3_3g2|mb3_3g3|2_4|1_5|4_2|5_1|6_0|1_4|2_3|3_2|4_1|5_0|1_6|2_5|3_4|4_3|5_2|6_1|7_0|1_7) echo "--params $1 --steps 2 --warmup 1" ;;
    *) echo "--params $1 --steps 5 --warmup 1" ;;
  esac
}
STAGES=${STAGES:-"tests smoke bench"}
for s in $STAGES; do
  case $s in
    tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    tests:*) step gpu_tests_${s#tests:} 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${s#tests:}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 900 python -u bench.py ;;
    bench:*) step bench_${s#bench:} 600 python -u bench.py $(kargs ${s#bench:}) ;;
    # sct:<VAR>=<value>: the single-ciphertext calling-pattern probe under one coalescer setting
    # (several settings: VAR=v,VAR2=w; probe arguments from $SCT_ARGS)
    sct:*) kv=${s#sct:}; step sct_${kv//[=,]/_} 300 env ${kv//,/ } python -u scripts/single_ct_probe.py $SCT_ARGS ;;
    # ab:<tag>:<VAR>=<value>: the bench of <tag> under one engine environment switch (A/B)
    ab:*) r=${s#ab:}; t=${r%%:*}; kv=${r#*:}; step ab_${t}_${kv//=/_} 600 env "$kv" python -u bench.py $(kargs $t) --no-cpu-baseline --no-host-abi ;;
    # the N = 32768, L = 2 CMUX through the split path instead of the grouped one (A/B)
    splitab:*) step splitab_${s#splitab:} 600 env TFHE_MI355_LARGE_SPLIT=1 python -u bench.py $(kargs ${s#splitab:}) --no-cpu-baseline --no-host-abi ;;
    kstats:*) t=${s#kstats:}; step kstats_$t 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kstats_$t -o run \
                --output-format csv -- python3 bench.py $(kargs $t) --no-cpu-baseline --no-host-abi ;;
    pmc:*) t=${s#pmc:}; step pmc_$t 1100 bash scripts/pmc_workload.sh $t ;;
    # two ranks sharing the box's one GPU over gloo: the multi-rank default run (every
    # configuration merged into one line), as the driver's N-GPU run executes it
    rehearse2) step rehearse2 900 env BENCH_DIST_BACKEND=gloo python -u bench.py --gpus 2 --steps 5 --warmup 1 ;;
  esac
done

#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash/timeout (rc not 0/1) stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STAGES=${STAGES:-"tests smoke bench prof"}
for s in $STAGES; do
  case $s in
    tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps 5 --warmup 1 ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --params 2_2 --steps 5 --warmup 1 --no-cpu-baseline --no-host-abi ;;
    benchall) for prm in mb3 mb2 4_4 mul32; do step bench_$prm 600 python bench.py --params $prm --steps 3 --warmup 1; done ;;
    profmb)  step prof_mb3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mb3 -o run --output-format csv -- python3 bench.py --params mb3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi ;;
    prof44)  step prof_4_4 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_4_4 -o run --output-format csv -- python3 bench.py --params 4_4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi ;;
    pmc1)  step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc1 -o run --output-format csv -- python3 bench.py --params 2_2 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi ;;
    pmc2)  step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc2 -o run --output-format csv -- python3 bench.py --params 2_2 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi ;;
    pmc3)  step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD -d gpurun_out/pmc3 -o run --output-format csv -- python3 bench.py --params 2_2 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi ;;
  esac
done

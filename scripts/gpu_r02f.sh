#!/bin/bash
# round-2 GPU session F (HEAD after the persistent ticket queue): GPU suite, smoke, benches,
# kernel traces of 2_2 and 4_4
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r02f
mkdir -p $out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -2 "$out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
STAGES=${STAGES:-"tests smoke bench kt"}
for s in $STAGES; do
  case $s in
    tests) step gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench_2_2 400 python bench.py --steps 5 --warmup 1 ;;
    kt) for t in ${KT:-2_2 4_4}; do
          st=5; [ "$t" = 4_4 ] && st=2
          step kt_$t 400 rocprofv3 --kernel-trace --stats -d $out/kt_$t -o run --output-format csv -- \
            python3 bench.py --params $t --steps $st --warmup 1 --no-cpu-baseline --no-host-abi
        done ;;
  esac
done

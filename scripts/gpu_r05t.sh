#!/bin/bash
# round 5: two chunk lanes for the multi-bit split CMUX (TFHE_MI355_MB_LANES=2): the multi-bit split
# tests + goldens with the switch on, then an A/B at mb3_3g3 and mb3_3g2
set -o pipefail
mkdir -p gpurun_out
TFHE_MI355_MB_LANES=2 timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_golden.py -m gpu -v --timeout 300 --timeout-method thread \
    -k "multi_bit or golden" > gpurun_out/r05_lanes_tests.log 2>&1 || { tail -30 gpurun_out/r05_lanes_tests.log; exit 1; }
tail -3 gpurun_out/r05_lanes_tests.log
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel'), round(d['roofline']['kernel_ms'],4), d['check'])" "$1"; }
for p in mb3_3g3 mb3_3g2; do
  for v in 1 2 1 2; do
    TFHE_MI355_MB_LANES=$v timeout -k 10 200 python bench.py --params $p --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call \
      > gpurun_out/r05_lanes_${p}_v$v.json 2> gpurun_out/r05_lanes_${p}_v$v.log || exit 1
    show gpurun_out/r05_lanes_${p}_v$v.json
  done
done

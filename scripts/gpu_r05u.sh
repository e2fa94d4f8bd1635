#!/bin/bash
# round 5: two multi-bit chunk lanes with full-size chunks per lane (TFHE_MI355_LARGE_CHUNK = 2 x lane chunk)
set -o pipefail
mkdir -p gpurun_out
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel'), round(d['roofline']['kernel_ms'],4), d['check'])" "$1"; }
for c in 1024 768 1536; do
  for v in 2 1; do
    TFHE_MI355_LARGE_CHUNK=$c TFHE_MI355_MB_LANES=$v timeout -k 10 200 python bench.py --params mb3_3g3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call \
      > gpurun_out/r05_lanes2_c${c}_v$v.json 2> gpurun_out/r05_lanes2_c${c}_v$v.log || exit 1
    show gpurun_out/r05_lanes2_c${c}_v$v.json
  done
done

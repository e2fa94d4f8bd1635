#!/bin/bash
# round 5: multi-bit chunk sweep after the pair2 / fused changes (TFHE_MI355_LARGE_CHUNK), g3 and g2
set -o pipefail
mkdir -p gpurun_out
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), d['check'])" "$1"; }
for p in mb3_3g3 mb3_3g2; do
  for c in 512 768 1024 1280 2048 512 1024; do
    TFHE_MI355_LARGE_CHUNK=$c timeout -k 10 200 python bench.py --params $p --steps 3 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call \
      > gpurun_out/r05_mbchunk_${p}_c$c.json 2> gpurun_out/r05_mbchunk_${p}_c$c.log || exit 1
    show gpurun_out/r05_mbchunk_${p}_c$c.json
  done
done

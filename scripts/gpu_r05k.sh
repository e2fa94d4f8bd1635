#!/bin/bash
# round 5: 3_3 batch-size sweep, on-chip CMUX vs the digits-fed split CMUX (for the count switch)
set -o pipefail
mkdir -p gpurun_out
C=1,8,32,64,96,128,160,192,256,384,512
for v in 1 0; do
  LAT_PARAMS=PARAM_MESSAGE_3_CARRY_3_KS_PBS TFHE_MI355_ONCHIP=$v timeout -k 10 400 python scripts/latency_probe.py $C > gpurun_out/r05_sweep33_onchip$v.json 2> gpurun_out/r05_sweep33_onchip$v.log || { tail -5 gpurun_out/r05_sweep33_onchip$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], {k: round(v['ms'],2) for k,v in d['ms'].items()}, all(v['decrypt_ok']==int(k) for k,v in d['ms'].items()))" gpurun_out/r05_sweep33_onchip$v.json
done

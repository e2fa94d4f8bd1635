#!/bin/bash
# round 5: 3_3 on-chip CMUX, level-L GGSW prefetch before the forward FFT (4 / 8 slots) vs HEAD (same box)
set -o pipefail
mkdir -p gpurun_out
B="--params 3_3 --batch 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for pass in 1 2; do
for v in base pf08 prev; do
  lib=$PWD/tfhe-rs-odd_amd/lib/libtfhe_mi355.so; [ $v = base ] || lib=$PWD/tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so
  TFHE_MI355_LIB=$lib timeout -k 10 200 python bench.py $B > gpurun_out/r05_pf0_$v.json 2> gpurun_out/r05_pf0_$v.log || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel_times_ms'))" gpurun_out/r05_pf0_$v.json
done
done

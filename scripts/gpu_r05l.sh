#!/bin/bash
# round 5: large_mb_pair2_kernel timing-only ablations (MB2_TSKIP / PBS_MB_TSKIP_MONO; wrong outputs)
set -o pipefail
mkdir -p gpurun_out
B="--params mb3_3g3 --batch 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-host-abi --no-single-call"
for v in base m1 m2 m4 m8 m9 mm; do
  lib=$PWD/tfhe-rs-odd_amd/lib/libtfhe_mi355.so; [ $v = base ] || lib=$PWD/tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so
  TFHE_MI355_LIB=$lib timeout -k 10 200 python bench.py $B > gpurun_out/r05_mb2ts_$v.json 2> gpurun_out/r05_mb2ts_$v.log; rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), d['roofline'].get('kernel_times_ms'))" gpurun_out/r05_mb2ts_$v.json
done

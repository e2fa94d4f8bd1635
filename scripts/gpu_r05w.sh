#!/bin/bash
# round 5: a second copy of the classic Fourier key read by every other same-XCD workgroup
# (TFHE_MI355_BSK_COPIES=2, experiment): parity with the switch on, then an interleaved A/B at 2_2
set -o pipefail
mkdir -p gpurun_out
TFHE_MI355_BSK_COPIES=2 timeout -k 10 300 python -u -m pytest tests/test_pbs_gpu.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r05_bskcopies_tests.log 2>&1 || { tail -20 gpurun_out/r05_bskcopies_tests.log; exit 1; }
tail -2 gpurun_out/r05_bskcopies_tests.log
for v in 1 2 1 2 1 2; do
  TFHE_MI355_BSK_COPIES=$v timeout -k 10 200 python bench.py --params 2_2 --steps 10 --warmup 2 --no-cpu-baseline --no-host-abi --no-single-call --no-other-workloads \
    > gpurun_out/r05_bskcopies_v$v.json 2> gpurun_out/r05_bskcopies_v$v.log || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), round(d['roofline']['kernel_ms'],3), d['check'])" gpurun_out/r05_bskcopies_v$v.json
done

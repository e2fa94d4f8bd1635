#!/bin/bash
# config 3 at its full size at HEAD: 65,536 ciphertexts KS+PBS at N = 32768 in one call
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r02p
mkdir -p $out
timeout -k 10 600 python -u bench.py --params 4_4 --batch 65536 --steps 1 --warmup 0 --no-cpu-baseline --no-host-abi > $out/bench_4_4_full.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $out/bench_4_4_full.log | cut -c1-300; exit $rc

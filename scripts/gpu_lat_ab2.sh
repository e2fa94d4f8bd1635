#!/bin/bash
# latency-kernel A/B: variants built by scripts/build_variant.sh, two interleaved passes, counts 1 and 256
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
set -e
B=tfhe-rs-odd_amd/build
for pass in 1 2; do
  for v in ${VARIANTS:-base prio pref2 pp}; do
    lib=$B/$v/libtfhe_mi355.so; [ "$v" = base ] && lib=tfhe-rs-odd_amd/lib/libtfhe_mi355.so
    TFHE_MI355_LIB=$lib timeout -k 10 200 python scripts/latency_probe.py 1,256 > gpurun_out/ab_${v}_$pass.json 2> gpurun_out/ab_${v}_$pass.log
  done
done

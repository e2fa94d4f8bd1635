#!/bin/bash
# per-phase cycle stamps of the latency kernel (LAT_STAMPS=1 variant built by build_variant.sh stamps)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
LAT_STAMPS=1 TFHE_MI355_LIB=tfhe-rs-odd_amd/build/stamps/libtfhe_mi355.so timeout -k 10 200 \
  python scripts/latency_probe.py 1,256 > gpurun_out/${ROUND:-r04}_lat_stamps_${TAG:-map1}.json 2> gpurun_out/lat_stamps.log

#!/bin/bash
# timing-only: the 2_2 throughput kernel without its rotation gather (build/tskiprot, wrong outputs)
# vs the default build, two passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for pass in 1 2; do
  for v in base tskiprot; do
    lib=tfhe-rs-odd_amd/build/$v/libtfhe_mi355.so; [ "$v" = base ] && lib=tfhe-rs-odd_amd/lib/libtfhe_mi355.so
    TFHE_MI355_LIB=$lib timeout -k 10 200 python -u bench.py --params 2_2 --steps 5 --warmup 1 --no-cpu-baseline \
      --no-host-abi --no-single-call > gpurun_out/r04_cltskip_${v}_$pass.log 2>&1
    echo "bench $v $pass rc=$?"
  done
done

#!/bin/bash
# build_variant.sh NAME "EXTRA HIPFLAGS" -> tfhe-rs-odd_amd/build/NAME/libtfhe_mi355.so
set -e
cd "$(dirname "$0")/../tfhe-rs-odd_amd"
d=build/$1; mkdir -p $d
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $2"
for f in pbs_multibit.hip pbs_latency.hip; do  # as the Makefile
  hipcc $F ${MB_SCHED--mllvm -amdgpu-sched-strategy=max-ilp} -c -o $d/${f%.hip}.o csrc/$f &
done
for f in pbs_classic.hip pbs_large.hip keyswitch.hip lwe_ops.hip glwe_ops.hip csprng.hip; do hipcc $F -c -o $d/${f%.hip}.o csrc/$f & done
for f in capi.cpp client.cpp serde.cpp; do hipcc $F -c -o $d/${f%.cpp}.o csrc/$f & done
wait
hipcc $F -shared -o $d/libtfhe_mi355.so $d/*.o
echo built $d

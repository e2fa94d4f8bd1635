#!/bin/bash
# bv1.sh NAME "FLAGS": rebuild pbs_large.o with FLAGS, link with the Makefile's other objects
set -e
cd /root/repo/tfhe-rs-odd_amd
d=build/$1; mkdir -p $d
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function $2 -c -o $d/pbs_large.o csrc/pbs_large.hip 2>/dev/null
objs=$(ls build/*.o | grep -v pbs_large.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libtfhe_mi355.so $objs $d/pbs_large.o
echo built $d

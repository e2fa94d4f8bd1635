#!/bin/bash
# build_variant_obj.sh NAME SRC "FLAGS": rebuild csrc/SRC.hip's object with FLAGS into build/NAME and
# link it with the Makefile's other objects (A/B libraries: TFHE_MI355_LIB=.../build/NAME/libtfhe_mi355.so)
set -e
cd /root/repo/tfhe-rs-odd_amd
d=build/$1; mkdir -p $d
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function $3 -c -o $d/$2.o csrc/$2.hip 2>/dev/null
objs=$(ls build/*.o | grep -v "/$2.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libtfhe_mi355.so $objs $d/$2.o
echo built $d

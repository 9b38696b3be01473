#!/bin/bash
# usage: buildvar.sh name "flags"
set -e
cd /root/repo/sdface-gan_amd
n=$1; shift
mkdir -p build_var/$n lib_var/$n
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -fno-slp-vectorize $@ -c csrc/field_f16x3.hip -o build_var/$n/field_f16x3.o
objs=$(ls build/*.o | grep -v field_f16x3.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib_var/$n/libsdfr.so $objs build_var/$n/field_f16x3.o
echo built $n

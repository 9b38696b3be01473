#!/bin/bash
# Build libsdfr.so variants that differ only in field_f16x3.hip compile-time
# options, into sdface-gan_amd/lib_var/<name>/ (profiling aid; SDFR_LIB selects one).
#   scripts/build_variants.sh name1 "-DFOO=1" name2 "-DFOO=0 -DBAR=1" ...
set -eu
cd "$(dirname "$0")/../sdface-gan_amd"
make -s build/encoders.o build/render_ngp.o build/decoder.o build/conv_f16x3.o
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall"
pids=()
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p lib_var/$name
  ( /opt/rocm/bin/hipcc $FLAGS $defs -c csrc/field_f16x3.hip -o lib_var/$name/field_f16x3.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib_var/$name/libsdfr.so \
        build/encoders.o build/render_ngp.o lib_var/$name/field_f16x3.o build/decoder.o build/conv_f16x3.o &&
    echo "built $name ($defs)" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done

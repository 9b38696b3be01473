#!/bin/bash
# Build libsdfr.so variants that differ only in one source's compile-time options
# (VAR_SRC = field_f16x3 (default) or conv_f16x3), into sdface-gan_amd/lib_var/<name>/
# (profiling aid; SDFR_LIB selects one).
#   [VAR_SRC=conv_f16x3] scripts/build_variants.sh name1 "-DFOO=1" name2 "-DFOO=0 -DBAR=1" ...
set -eu
cd "$(dirname "$0")/../sdface-gan_amd"
SRC=${VAR_SRC:-field_f16x3}
VD=${VAR_DIR:-lib_var}
ALL="encoders render_ngp field_f16x3 decoder conv_f16x3 mesh linear_f16x3 linear_head"
FIXED=""
for s in $ALL; do [ "$s" = "$SRC" ] || FIXED="$FIXED build/$s.o"; done
make -s $FIXED
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall"
[ "$SRC" = field_f16x3 ] && FLAGS="$FLAGS -fno-slp-vectorize"   # as the Makefile
pids=()
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p $VD/$name
  ( /opt/rocm/bin/hipcc $FLAGS $defs -c csrc/$SRC.hip -o $VD/$name/$SRC.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $VD/$name/libsdfr.so \
        $FIXED $VD/$name/$SRC.o &&
    echo "built $name ($defs)" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done

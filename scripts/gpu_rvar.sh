#!/bin/bash
set -u
mkdir -p gpurun_out
ARGS=""
for v in ${VARS}; do ARGS="$ARGS sdface-gan_amd/lib_var/$v/libsdfr.so@r"; done
REPS=${REPS:-3} timeout -k 10 500 python scripts/field_time.py sdface-gan_amd/lib/libsdfr.so@p $ARGS > gpurun_out/ft_rvar.log 2>&1
rc=$?; echo "ft rc=$rc"; grep SUMMARY gpurun_out/ft_rvar.log
exit $rc

#!/bin/bash
# field_r_kernel ablations: field-stage time and (one counter pass each) clock + MFMA busy
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
V="rbase rnoaread rnoside rnodma rnobar"
ARGS=""
for v in $V; do ARGS="$ARGS sdface-gan_amd/lib_var/$v/libsdfr.so@r"; done
REPS=3 timeout -k 10 400 python scripts/field_time.py $ARGS > gpurun_out/ft_rabl.log 2>&1
rc=$?; echo "ft rc=$rc"; grep SUMMARY gpurun_out/ft_rabl.log
[ $rc -eq 0 ] || exit $rc
for v in $V; do
  SDFR_FIELD_KERNEL=r SDFR_LIB=$R/sdface-gan_amd/lib_var/$v/libsdfr.so timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "field_r_kernel" --output-format csv \
      -d "$R/gpurun_out/pmc_abl_$v" -o "c" -- python3 "$R/scripts/render_only.py" f16x3 > "gpurun_out/pmc_abl_$v.log" 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

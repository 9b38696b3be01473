#!/bin/bash
# SQ counter passes on the field kernels: NETS="ngp siren" (ngp -> field_r_kernel<NgpNet>,
# siren -> field_p_kernel<SirenNet>); SDFR_LIB selects a variant build (scripts/build_variants.sh).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS"
TAG=${TAG:-}
for net in ${NETS:-ngp siren}; do
  if [ $net = ngp ]; then k=field_r_kernel; else k=field_p_kernel; fi
  for pass in 1 2; do
    if [ $pass = 1 ]; then PMC=$P1; else PMC=$P2; fi
    timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "$k" --output-format csv \
        -d "$R/gpurun_out/pmc_${net}${TAG}$pass" -o "f$pass" -- python3 "$R/scripts/render_only.py" f16x3 $net \
        > "gpurun_out/pmc_${net}${TAG}$pass.log" 2>&1
    rc=$?; echo "pmc $net$TAG$pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done

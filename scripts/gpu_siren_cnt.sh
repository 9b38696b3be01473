#!/bin/bash
# SQ / GRBM counter passes on the SIREN field kernel (configs[4]'s generator)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS"
for n in 1 2; do
  eval PMC=\$P$n
  timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "field_p_kernel" --output-format csv \
      -d "$R/gpurun_out/pmc_sfield_sq$n" -o "sfield_sq$n" -- python3 "$R/scripts/render_only.py" f16x3 siren \
      > "gpurun_out/pmc_sfield_sq$n.log" 2>&1
  rc=$?; echo "sfield_sq$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

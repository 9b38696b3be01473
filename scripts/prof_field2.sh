#!/bin/bash
# Field-kernel diagnosis on the GPU: ablation timings (lib_abl) for the selected
# kernel generation (SDFR_FIELD_KERNEL, default 2) and its SQ counter passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
SDFR_LIB=sdface-gan_amd/lib_abl/libsdfr.so timeout -k 10 300 python scripts/field_ablation.py f16x3 \
    > gpurun_out/ablation.log 2>&1
rc=$?; echo "ablation rc=$rc"; grep -E "variant" gpurun_out/ablation.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS"

  timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex field_x --output-format csv \
      -d "$R/gpurun_out/pmc_f${PASS_TAG:-}sq1" -o sq1 -- python3 "$R/scripts/render_only.py" f16x3 \
      > gpurun_out/pmc_sq1.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-include-regex field_x --output-format csv \
      -d "$R/gpurun_out/pmc_f${PASS_TAG:-}sq2" -o sq2 -- python3 "$R/scripts/render_only.py" f16x3 \
      > gpurun_out/pmc_sq2.log 2>&1 || exit $?


echo counters-done

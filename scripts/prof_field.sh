#!/bin/bash
# Field-kernel diagnosis: ablation timings + SQ counter passes on the renderer only.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
PREC=${1:-f16x3}
SDFR_LIB=sdface-gan_amd/lib_abl/libsdfr.so timeout -k 10 300 python scripts/field_ablation.py $PREC \
    > gpurun_out/ablation.log 2>&1
rc=$?; echo "ablation rc=$rc"; grep -v amdgpu.ids gpurun_out/ablation.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS --kernel-include-regex field --output-format csv -d "$R/gpurun_out/prof_sq1" -o sq1 \
    -- python3 "$R/scripts/render_only.py" $PREC > gpurun_out/prof_sq1.log 2>&1
rc=$?; echo "sq1 rc=$rc"; tail -2 gpurun_out/prof_sq1.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --kernel-include-regex field --output-format csv -d "$R/gpurun_out/prof_sq2" -o sq2 \
    -- python3 "$R/scripts/render_only.py" $PREC > gpurun_out/prof_sq2.log 2>&1
rc=$?; echo "sq2 rc=$rc"; tail -2 gpurun_out/prof_sq2.log
exit $rc

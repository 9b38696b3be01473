#!/bin/bash
# SQ / GRBM counter passes on field_x2_kernel (SDFR_FIELD_X2=1) and field_p_kernel
# (render_only.py), one rocprofv3 --pmc pass per counter group.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name regex cmd...
    local name=$1 rx=$2; shift 2
    timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "$rx" --output-format csv \
        -d "$R/gpurun_out/pmc_$name" -o "$name" -- "$@" > "gpurun_out/pmc_$name.log" 2>&1
    local rc=$?; echo "$name rc=$rc"; return $rc
}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS"
PMC=$P1 run p_sq1 field_p_kernel python3 "$R/scripts/render_only.py" f16x3 &&
PMC=$P2 run p_sq2 field_p_kernel python3 "$R/scripts/render_only.py" f16x3 &&
export SDFR_FIELD_X2=1 &&
PMC=$P1 run x2_sq1 field_x2_kernel python3 "$R/scripts/render_only.py" f16x3 &&
PMC=$P2 run x2_sq2 field_x2_kernel python3 "$R/scripts/render_only.py" f16x3

#!/bin/bash
# SQ / GRBM counter passes (rocprofv3 --pmc, one pass per counter group, each under
# its own time limit) on the field kernel (render_only.py) and the decoder
# convolutions (decoder_only.py); summarised by scripts/summarize_counters.py.
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
FIELD=${FIELD_PREC:-f16x3}
PMC=$P1 run field_sq1 field_r_kernel python3 "$R/scripts/render_only.py" $FIELD &&
PMC=$P2 run field_sq2 field_r_kernel python3 "$R/scripts/render_only.py" $FIELD &&
PMC=$P1 run conv_sq1 "conv_[xh]_kernel" python3 "$R/scripts/decoder_only.py" &&
PMC=$P2 run conv_sq2 "conv_[xh]_kernel" python3 "$R/scripts/decoder_only.py"

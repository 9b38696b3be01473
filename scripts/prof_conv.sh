#!/bin/bash
# Decoder-conv diagnosis: per-layer timings (+ variants given as args) and SQ counter
# passes on conv_x_kernel over the five decoder layer shapes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/conv_time.py "$@" > gpurun_out/conv_time.log 2>&1
rc=$?; echo "conv_time rc=$rc"; grep -v amdgpu.ids gpurun_out/conv_time.log
[ $rc -eq 0 ] || exit $rc
[ -n "${NO_PMC:-}" ] && exit 0
export TMPDIR=/tmp REPS=2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS --kernel-include-regex conv_x --output-format csv -d "$R/gpurun_out/prof_csq1" -o sq1 \
    -- python3 "$R/scripts/conv_time.py" > gpurun_out/prof_csq1.log 2>&1
rc=$?; echo "sq1 rc=$rc"; tail -2 gpurun_out/prof_csq1.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS --kernel-include-regex conv_x --output-format csv -d "$R/gpurun_out/prof_csq2" -o sq2 \
    -- python3 "$R/scripts/conv_time.py" > gpurun_out/prof_csq2.log 2>&1
rc=$?; echo "sq2 rc=$rc"; tail -2 gpurun_out/prof_csq2.log
exit $rc

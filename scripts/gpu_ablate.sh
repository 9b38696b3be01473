#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/field_ablation.py > gpurun_out/ablation.log 2>&1
rc=$?; echo "ablation rc=$rc"; cat gpurun_out/ablation.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$R/gpurun_out/prof_sq" -o sq \
    -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_sq.log 2>&1
rc=$?; echo "sq rc=$rc"; tail -3 gpurun_out/prof_sq.log
timeout -k 10 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d "$R/gpurun_out/prof_sq2" -o sq2 \
    -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_sq2.log 2>&1
rc=$?; echo "sq2 rc=$rc"; tail -3 gpurun_out/prof_sq2.log
exit 0

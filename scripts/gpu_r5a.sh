#!/bin/bash
# round 5: new GPU tests (fc fused renderer, RCCL world 1), then field-kernel ablation timings
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
SDFR_PARITY_JSON=gpurun_out/parity_fc.json timeout -k 10 900 python -u -m pytest -v --timeout 200 \
    --timeout-method thread tests/test_gpu_fc.py tests/test_gpu_linear.py tests/test_gpu_stage1.py tests/test_gpu_render.py tests/test_gpu_train.py > gpurun_out/fc.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" gpurun_out/fc.log | tail -8; cat gpurun_out/parity_fc.json 2>/dev/null | head -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py \
    > gpurun_out/rccl.log 2>&1; rc2=$?
tail -5 gpurun_out/rccl.log
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
REPS=3 bash scripts/gpu_var.sh

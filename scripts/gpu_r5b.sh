#!/bin/bash
# round 5: parity after the field_r DMA spread + fc / DDP test fixes, then A/B timings
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
SDFR_PARITY_JSON=gpurun_out/parity_b.json timeout -k 10 900 python -u -m pytest -v --timeout 300 \
    --timeout-method thread -s tests/test_gpu_fc.py tests/test_gpu_render.py tests/test_gpu_train.py \
    -k "fc or render or stage1_ddp" > gpurun_out/b.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|varying" gpurun_out/b.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
REPS=3 bash scripts/gpu_var.sh

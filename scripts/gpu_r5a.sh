#!/bin/bash
# round 5: field-kernel ablation timings + the RCCL world-1 tests
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
REPS=3 bash scripts/gpu_var.sh || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py \
    > gpurun_out/rccl.log 2>&1; rc=$?
tail -5 gpurun_out/rccl.log; exit $rc

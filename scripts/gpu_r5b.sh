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
timeout -k 10 400 python scripts/conv_time.py sdface-gan_amd/lib/libsdfr.so sdface-gan_amd/lib_cvar/*/libsdfr.so \
    > gpurun_out/conv_var.txt 2>&1; echo "conv_time rc=$?"; grep -E "lib|total|T " gpurun_out/conv_var.txt | head -60

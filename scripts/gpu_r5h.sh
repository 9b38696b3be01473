#!/bin/bash
# round 5: conv_t edge split-K: parity, B=32 trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_decoder.py \
    tests/test_gpu_render.py -k "conv or decoder or generator" > gpurun_out/h.log 2>&1; rc=$?
tail -2 gpurun_out/h.log; grep FAILED gpurun_out/h.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/conv_time.py > gpurun_out/conv_h5.txt 2>&1; grep -E " T |total" gpurun_out/conv_h5.txt
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_trace5" -o trace \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/prof_trace5.log 2>&1
echo "trace rc=$?"; tail -1 gpurun_out/prof_trace5.log | cut -c1-200

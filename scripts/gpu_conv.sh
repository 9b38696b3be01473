#!/bin/bash
# decoder convolution A/B: parity of the conv + decoder tests, then timings of each
# library given (default: the in-tree one) at the bench's layer shapes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_decoder.py -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/conv_act_time.py "$@" && timeout -k 10 300 python scripts/conv_time.py "$@"

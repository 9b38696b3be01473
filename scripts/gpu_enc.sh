#!/bin/bash
# gather A/B: encoder + render parity, then encode_time.py for each library given
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_encoders.py tests/test_gpu_render.py -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_enc.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_enc.log; [ $rc -eq 0 ] || exit $rc
for l in "$@"; do
  echo "$l"; SDFR_LIB=$l timeout -k 10 200 python scripts/encode_time.py 289 || exit 1
done

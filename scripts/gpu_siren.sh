#!/bin/bash
# SIREN renderer: render + stage-1 GPU tests, then field timing (NET=siren) of the
# libraries given
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_stage1.py tests/test_gpu_mesh.py -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_siren.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_siren.log; [ $rc -eq 0 ] || exit $rc
NET=siren timeout -k 10 300 python scripts/field_time.py "$@"

#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mesh.py -x -q -p no:cacheprovider \
    --timeout 180 --timeout-method thread > gpurun_out/pytest_mesh.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_mesh.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_mesh.py > gpurun_out/bench_mesh.log 2>&1
rc=$?; echo "bench_mesh rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_mesh.log | tail -4
exit $rc

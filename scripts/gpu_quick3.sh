#!/bin/bash
# Render + mesh + encoder parity, then a short bench (no CPU baseline / extras), 3 runs
set -u
mkdir -p gpurun_out
export SDFR_PARITY_JSON=gpurun_out/parity_q3.json
timeout -k 10 500 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_mesh.py tests/test_gpu_encoders.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_q3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_q3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/bench_q3_$i.log 2>&1 || exit $?
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/bench_q3_$i.log').read().strip().splitlines()[-1])
print('bench', round(d['value'],1), 'ms', round(d['ms_per_step'],3), 'field', round(d['stage_ms_per_step']['field'],3), 'grid', round(d['stage_ms_per_step']['hash_grid'],4), 'gather frac', round(d['roofline_gather']['frac'],3), 'field frac', round(d['roofline']['frac'],3))"
done

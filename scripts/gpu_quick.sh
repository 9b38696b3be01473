#!/bin/bash
# Quick GPU iteration: render parity tests (both field precisions) + bench of each.
set -u
mkdir -p gpurun_out
export SDFR_PARITY_JSON=gpurun_out/parity.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_render.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_render.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for prec in f16x3 fp32; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --field-precision $prec \
      > gpurun_out/bench_$prec.log 2>&1
  rc=$?; echo "bench $prec rc=$rc"; tail -2 gpurun_out/bench_$prec.log
  [ $rc -eq 0 ] || exit $rc
done

#!/bin/bash
# decoder tests (incl. split-fp16 conv) + render tests + bench (f16x3)
set -u
mkdir -p gpurun_out
export SDFR_PARITY_JSON=gpurun_out/parity.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_render.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_dec.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_dec.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_dec.log | cut -c1-400
exit $rc

#!/bin/bash
# Quick GPU check: selected parity tests + field-stage timing (+ optional bench).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export SDFR_PARITY_JSON=$R/gpurun_out/parity_quick.json
rm -f "$SDFR_PARITY_JSON"
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_render.py tests/test_gpu_encoders.py} \
    -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -x \
    > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_quick.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/field_time.py ${LIBS:-sdface-gan_amd/lib/libsdfr.so} 2>&1 | tee gpurun_out/field_time.log
rc=$?; [ $rc -eq 0 ] || exit $rc
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_quick.log | cut -c1-600
fi
exit $rc

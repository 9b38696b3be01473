#!/bin/bash
# GPU session: parity tests, bench, rocprofv3 kernel trace + PMC traffic passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export SDFR_PARITY_JSON=$R/gpurun_out/parity.json
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_trace" -o trace \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/prof_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof_fetch" -o fetch \
    -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/prof_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/prof_write" -o write \
    -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/prof_write.log 2>&1
rc=$?; echo "write rc=$rc"
find gpurun_out -name "*.csv" | head -20
exit $rc

#!/bin/bash
# One GPU session: parity tests, then (if nothing faulted) a short bench and a
# rocprofv3 kernel-trace summary.  Stops at the first fault / abort / timeout.
set -u
mkdir -p gpurun_out
export SDFR_PARITY_JSON=gpurun_out/parity.json
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc

#!/bin/bash
# GPU session: the -m gpu parity suite (parity record -> gpurun_out/parity.json).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export SDFR_PARITY_JSON=$R/gpurun_out/parity.json
rm -f "$SDFR_PARITY_JSON"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -30
exit $rc

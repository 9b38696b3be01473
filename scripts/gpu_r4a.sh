#!/bin/bash
# Round 4: field_q parity + A/B, SIREN double-backward / DDP tests, linear tests
set -u
mkdir -p gpurun_out
export SDFR_PARITY_JSON=gpurun_out/parity_r4a.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_stage1.py tests/test_gpu_linear.py tests/test_gpu_encoders.py \
    "tests/test_gpu_train.py::test_stage1_ddp_gradients_equal_single_process" "tests/test_gpu_train.py::test_stage1_step_64" \
    -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_r4a.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_r4a.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_q.sh

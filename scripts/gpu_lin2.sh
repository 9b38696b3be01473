#!/bin/bash
# GPU session: training-GEMM tests, stage-1 bench, stage-1 kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear.py ${EXTRA_TESTS:-} -m gpu -q -x \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_lin.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_lin.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/train_bench.py --stage 1 --steps 8 --warmup 3 \
    > gpurun_out/train1.json 2> gpurun_out/train1.err
r=$?; echo "train rc=$r"; tail -1 gpurun_out/train1.json; [ $r -eq 0 ] || exit $r
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_train1" -o t1 \
    -- python3 "$R/scripts/train_bench.py" --stage 1 --steps 4 --warmup 2 > gpurun_out/prof_train1.log 2>&1
echo "prof rc=$?"

#!/bin/bash
# GPU session: training-GEMM kernels (tests, stage-1 bench both ways, kernel trace).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_stage1.py tests/test_gpu_train.py tests/test_gpu_encoders.py -m gpu -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_lin.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_lin.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for cfg in "torch 8" "f16x3 8"; do
  set -- $cfg
  timeout -k 10 300 python scripts/train_bench.py --stage 1 --steps 8 --warmup 3 --train-gemm $1 \
      --coord-pad $2 > gpurun_out/train1_$1_$2.json 2> gpurun_out/train1_$1_$2.err
  r=$?; echo "train $cfg rc=$r"; tail -1 gpurun_out/train1_$1_$2.json; [ $r -eq 0 ] || exit $r
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_train1" -o t1 \
    -- python3 "$R/scripts/train_bench.py" --stage 1 --steps 4 --warmup 2 > gpurun_out/prof_train1.log 2>&1
echo "prof rc=$?"
exit $rc

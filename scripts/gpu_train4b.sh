#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stage1.py tests/test_gpu_linear.py "tests/test_gpu_train.py::test_stage1_ddp_gradients_equal_single_process" "tests/test_gpu_train.py::test_stage1_step_64" -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_t4b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_t4b.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  timeout -k 10 300 python scripts/train_bench.py --stage 1 --net ngp --steps 8 --warmup 4 > gpurun_out/tb4b_ngp_$i.json 2> gpurun_out/tb4b_ngp_$i.err || exit $?
  tail -1 gpurun_out/tb4b_ngp_$i.json | cut -c1-150
done
timeout -k 10 300 python scripts/train_prof.py --net ngp --out gpurun_out/train4b_prof_ngp.txt > /dev/null 2>&1; echo "prof ngp rc=$?"

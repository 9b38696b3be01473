#!/bin/bash
# SIREN stage 1 with the second-order FiLM op: stage-1 / linear / DDP GPU tests, then
# SIREN stage-1 throughput (x2) and a torch.profiler pass
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stage1.py tests/test_gpu_linear.py "tests/test_gpu_train.py::test_stage1_ddp_gradients_equal_single_process" -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_t4c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_t4c.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python scripts/train_bench.py --stage 1 --net siren --steps 6 --warmup 3 > gpurun_out/tb4c_siren_$i.json 2> gpurun_out/tb4c_siren_$i.err || exit $?
  tail -1 gpurun_out/tb4c_siren_$i.json | cut -c1-150
done
timeout -k 10 300 python scripts/train_prof.py --net siren --out gpurun_out/train4c_prof_siren.txt > /dev/null 2>&1; echo "prof siren rc=$?"

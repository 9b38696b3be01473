#!/bin/bash
# round 5: conv_t_kernel parity (decoder tests + generator golden), then A/B timings
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_decoder.py \
    tests/test_gpu_render.py -k "conv or decoder or generator" > gpurun_out/d.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/d.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/conv_time.py > gpurun_out/conv_t.txt 2>&1; echo "conv_t rc=$?"
SDFR_CONV_T=0 timeout -k 10 300 python scripts/conv_time.py > gpurun_out/conv_x.txt 2>&1; echo "conv_x rc=$?"
grep -E " T |total" gpurun_out/conv_t.txt gpurun_out/conv_x.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/bench_t.log 2>&1
echo "bench rc=$?"; tail -1 gpurun_out/bench_t.log | cut -c1-250
SDFR_CONV_T=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/bench_x.log 2>&1
echo "bench x rc=$?"; tail -1 gpurun_out/bench_x.log | cut -c1-250

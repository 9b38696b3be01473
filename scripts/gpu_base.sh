#!/bin/bash
# Baseline on a fresh box: bench (no CPU baseline) + field-stage time of the product library.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras \
    > gpurun_out/bench_base.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_base.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
REPS=3 timeout -k 10 300 python scripts/field_time.py sdface-gan_amd/lib/libsdfr.so > gpurun_out/ft_base.log 2>&1
rc=$?; echo "ft rc=$rc"; tail -2 gpurun_out/ft_base.log
exit $rc

#!/bin/bash
# round 5: conv_t K split + mapping preload: parity, then B=1 trace and bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_decoder.py \
    tests/test_gpu_render.py > gpurun_out/g.log 2>&1; rc=$?
tail -3 gpurun_out/g.log; grep FAILED gpurun_out/g.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_b1g" -o b1 \
    -- python3 "$R/bench.py" --batch 1 --steps 30 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/prof_b1g.log 2>&1
echo "b1 trace rc=$?"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_g.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_g.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['extras'])"

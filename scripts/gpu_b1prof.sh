#!/bin/bash
# eval.py's own call (one face per Generator.forward): bench at B = 1 (eager) and its
# rocprofv3 kernel trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --batch 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extras \
    > gpurun_out/bench_b1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_b1" -o b1 \
    -- python3 "$R/bench.py" --batch 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extras \
    > gpurun_out/prof_b1.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc

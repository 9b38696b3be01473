#!/bin/bash
# rocprofv3 kernel trace of a short bench run -> gpurun_out/prof_t/ (args passed to bench.py)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_t" -o t \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/prof_t.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 gpurun_out/prof_t.log | cut -c1-200
exit $rc

#!/bin/bash
# L2 / L1 counters of conv_x_kernel over the five decoder layer shapes (one pass each).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp REPS=2
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-include-regex conv_x --output-format csv -d "$R/gpurun_out/prof_cmem" -o mem \
    -- python3 "$R/scripts/conv_time.py" "$@" > gpurun_out/prof_cmem.log 2>&1
rc=$?; echo "mem rc=$rc"; tail -3 gpurun_out/prof_cmem.log
exit $rc

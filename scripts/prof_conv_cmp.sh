#!/bin/bash
# L1/L2 counters of conv_x_kernel for each library given (one PMC pass per library).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp REPS=2
i=0
for lib in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --kernel-include-regex conv_x --output-format csv -d "$R/gpurun_out/prof_cmp$i" -o c \
      -- python3 "$R/scripts/conv_time.py" "$lib" > gpurun_out/prof_cmp$i.log 2>&1
  rc=$?; echo "$lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done

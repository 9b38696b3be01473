#!/bin/bash
# round 5: B = 1 transposed convs: strip kernel vs conv_t (unsplit, K split) with a kernel trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5m; mkdir -p $O
export TMPDIR=/tmp
for env in 1 2 3; do
  B=1 REPS=20 SDFR_CONV_T=$env timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/t$env" -o t \
     -- python3 scripts/conv_time.py > $O/ct$env.txt 2>&1 || exit 1
  echo "env $env"; grep -E " T |total" $O/ct$env.txt
done

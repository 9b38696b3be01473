#!/bin/bash
# round-end rehearsal: smoke() and the driver's default bench command (no flags)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5smoke; mkdir -p $O
s=$(date +%s)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log; echo "smoke $(( $(date +%s) - s )) s"; s=$(date +%s)
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-160; echo "bench $(( $(date +%s) - s )) s"

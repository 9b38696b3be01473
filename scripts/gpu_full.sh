#!/bin/bash
# Full GPU session: parity suite (parity record), smoke, then the bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
bash scripts/gpu_tests.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?; echo "smoke rc=$src"; tail -2 gpurun_out/smoke.log; [ $src -eq 0 ] || exit $src
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
brc=$?; echo "bench rc=$brc"; tail -1 gpurun_out/bench.log | cut -c1-400
exit $((rc > brc ? rc : brc))

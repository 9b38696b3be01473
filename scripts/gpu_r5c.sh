#!/bin/bash
# round 5 mid-round measurement: bench (ngp headline, siren, fc), kernel trace, SQ counters
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
for net in siren fc; do
  timeout -k 10 400 python bench.py --net $net --steps 10 --warmup 3 --no-extras --cpu-seconds 8 \
      > gpurun_out/bench_$net.log 2>&1
  rc=$?; echo "bench $net rc=$rc"; tail -1 gpurun_out/bench_$net.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_trace" -o trace \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/prof_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/prof_counters.sh
NETS="siren" TAG=r5 bash scripts/gpu_cnt.sh

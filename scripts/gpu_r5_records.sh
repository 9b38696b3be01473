#!/bin/bash
# round-5 records on one box: the bench lines (ngp default with the CPU baseline and
# extras, siren, fc, B = 1) and the rocprofv3 kernel traces of the B = 32 and B = 1
# commands, so every committed summary agrees with the bench line it sits beside
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5rec; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-120
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_trace" -o trace \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/prof_trace.log 2>&1 || exit 1
echo "trace ok"
timeout -k 10 300 python bench.py --net siren --steps 10 --warmup 3 --no-extras > $O/bench_siren.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --net fc --steps 10 --warmup 3 --no-extras > $O/bench_fc.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --batch 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_b1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_b1" -o b1 \
    -- python3 "$R/bench.py" --batch 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $O/prof_b1.log 2>&1 || exit 1
echo "b1 trace ok"

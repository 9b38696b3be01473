#!/bin/bash
# round-5 final: the whole GPU suite (parity record), bench lines (ngp default with the
# CPU baseline and extras, siren, fc, B = 1 + its kernel trace), mesh and training benches
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5final; mkdir -p $O
export SDFR_PARITY_JSON=$R/$O/parity.json TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 300 python bench.py --net siren --steps 10 --warmup 3 --no-extras > $O/bench_siren.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --net fc --steps 10 --warmup 3 --no-extras > $O/bench_fc.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --batch 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_b1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_b1" -o b1 \
    -- python3 "$R/bench.py" --batch 1 --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $O/prof_b1.log 2>&1
echo "b1 trace rc=$?"
timeout -k 10 300 python scripts/bench_mesh.py > $O/bench_mesh.log 2>&1; echo "mesh rc=$?"
timeout -k 10 400 python scripts/train_bench.py --stage 2 > $O/train2.log 2>&1; echo "train2 rc=$?"
timeout -k 10 400 python scripts/train_bench.py --stage 1 --net ngp > $O/train1_ngp.log 2>&1; echo "train1 ngp rc=$?"
timeout -k 10 400 python scripts/train_bench.py --stage 1 --net siren > $O/train1_siren.log 2>&1; echo "train1 siren rc=$?"
timeout -k 10 400 python scripts/train_bench.py --stage 1 --net fc > $O/train1_fc.log 2>&1; echo "train1 fc rc=$?"

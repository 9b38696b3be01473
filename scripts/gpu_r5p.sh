#!/bin/bash
# round 5: ToRGB weight product in the conv epilogue (ABI 10) + split-K bound 320: parity, B = 1 / 32 benches
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5p; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py \
    tests/test_gpu_render.py tests/test_gpu_train.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
for rep in 1 2; do
  timeout -k 10 200 python bench.py --batch 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/b1.log 2>&1 || { tail -5 $O/b1.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('$O/b1.log') if l.startswith('{')][-1])
print('b1', round(d['value'],1), 'graph', round(d['extras']['faces_per_s_b1_graph'],1), 'b8', round(d['extras']['faces_per_s_b8'],1))"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/b32.log 2>&1 || { tail -5 $O/b32.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('$O/b32.log') if l.startswith('{')][-1])
print('b32', round(d['value'],1), d['ms_per_step'])"
done

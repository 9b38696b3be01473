#!/bin/bash
# round 5: split-NHWC modulated features from the field kernel (ABI 12): parity, bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_render.py \
    tests/test_gpu_fc.py tests/test_gpu_decoder.py tests/test_gpu_mesh.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print('b32', round(d['value'],1), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'gather', round(d['roofline_gather']['frac'],3), 'b1g', round(d['extras']['faces_per_s_b1_graph'],1), 'b1', round(d['extras']['faces_per_s_b1'],1), 'b8', round(d['extras']['faces_per_s_b8'],1))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/tr" -o tr \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/tr.log 2>&1; echo "trace rc=$?"

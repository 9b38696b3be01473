#!/bin/bash
# round 5: full GPU suite + smoke + bench after the small-kernel / ABI 10 / overlap changes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; grep FAILED $O/pytest_gpu.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print('b32', round(d['value'],1), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'gather', round(d['roofline_gather']['frac'],3), 'dec', round(d['roofline_decoder']['frac'],3), 'b1g', round(d['extras']['faces_per_s_b1_graph'],1), 'b1', round(d['extras']['faces_per_s_b1'],1), 'b8', round(d['extras']['faces_per_s_b8'],1), 'cpu', d['cpu_baseline']['value'])"

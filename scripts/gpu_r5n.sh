#!/bin/bash
# round 5: conv_h K split at small batches: parity, B = 1 bench (eager + graphed) A/B, B = 32 check
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py \
    tests/test_gpu_render.py -k "conv or decoder or generator" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
P=$R/sdface-gan_amd/lib/libsdfr.so; V=$R/sdface-gan_amd/lib_var/hs0/libsdfr.so
for rep in 1 2; do for lib in $P $V; do
  SDFR_LIB=$lib timeout -k 10 200 python bench.py --batch 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/b1.log 2>&1 || { tail -5 $O/b1.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('$O/b1.log') if l.startswith('{')][-1])
print(sys.argv[1][-28:], 'b1', round(d['value'],1), 'graph', round(d['extras']['faces_per_s_b1_graph'],1), 'b8', round(d['extras']['faces_per_s_b8'],1))" $lib
done; done
timeout -k 10 300 python scripts/conv_act_time.py $P $V $P $V > $O/cat.txt 2>&1; cat $O/cat.txt

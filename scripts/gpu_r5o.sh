#!/bin/bash
# round 5: split-K bound for the batch-1 strip convs (SDFR_KSPLIT_MAX): B = 1 graphed A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5o; mkdir -p $O
P=$R/sdface-gan_amd/lib/libsdfr.so; V=$R/sdface-gan_amd/lib_var
for rep in 1 2; do for lib in $P $V/k320/libsdfr.so $V/k384/libsdfr.so; do
  SDFR_LIB=$lib timeout -k 10 200 python bench.py --batch 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/b1.log 2>&1 || { tail -5 $O/b1.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('$O/b1.log') if l.startswith('{')][-1])
print(sys.argv[1][-28:], 'b1', round(d['value'],1), 'graph', round(d['extras']['faces_per_s_b1_graph'],1), 'b8', round(d['extras']['faces_per_s_b8'],1))" $lib
done; done
B=1 REPS=20 timeout -k 10 300 python scripts/conv_time.py $P $V/k320/libsdfr.so $V/k384/libsdfr.so > $O/ct.txt 2>&1; grep -E "libsdfr| T |total" $O/ct.txt

#!/bin/bash
# round 5: split-K edge classes of conv_t_kernel: parity, conv timing A/B, bench A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py \
    tests/test_gpu_render.py -k "conv or decoder or generator" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
P=$R/sdface-gan_amd/lib/libsdfr.so; V=$R/sdface-gan_amd/lib_var/es0/libsdfr.so
REPS=20 timeout -k 10 300 python scripts/conv_time.py $P $V $P $V > $O/ct.txt 2>&1; grep -E "libsdfr| T |total" $O/ct.txt
for rep in 1 2; do for lib in $P $V; do
  SDFR_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1])
print(sys.argv[1][-28:], round(d['value'],1), round(d['ms_per_step'],3))" $lib
done; done

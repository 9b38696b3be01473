#!/bin/bash
# round 5: conv_h held y stores (SDFR_HDEFER 2 default / 1 / 0): parity + conv_act_time + bench A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5x; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py \
    tests/test_gpu_render.py -k "conv or decoder or generator" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
P=sdface-gan_amd/lib/libsdfr.so; V0=sdface-gan_amd/lib_var/hd0/libsdfr.so; V1=sdface-gan_amd/lib_var/hd1/libsdfr.so
timeout -k 10 400 python scripts/conv_act_time.py $P $V0 $V1 $P $V0 $V1 $P $V0 $V1 > $O/cat.txt 2>&1; cat $O/cat.txt
for L in $P $V0 $P $V0; do
  SDFR_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/b.txt 2>&1 || exit 1
  echo "$L $(tail -1 $O/b.txt | cut -c1-120)"
done

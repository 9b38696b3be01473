#!/bin/bash
# round 5: conv_h epilogue on packed fp32 (SDFR_HEPK): parity + conv_act_time A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py \
    tests/test_gpu_render.py -k "conv or decoder or generator" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
P=sdface-gan_amd/lib/libsdfr.so; V=sdface-gan_amd/lib_var/hp0/libsdfr.so
timeout -k 10 400 python scripts/conv_act_time.py $P $V $P $V $P $V > $O/cat.txt 2>&1; cat $O/cat.txt

#!/bin/bash
# round 5: conv_h / conv_t epilogue store shape + counted store waits: parity + timing
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_decoder.py \
    tests/test_gpu_render.py -k "conv or decoder or generator" > gpurun_out/k_t.txt 2>&1 || { tail -30 gpurun_out/k_t.txt; exit 1; }
tail -1 gpurun_out/k_t.txt
V=sdface-gan_amd/lib_var; P=sdface-gan_amd/lib/libsdfr.so
timeout -k 10 400 python scripts/conv_act_time.py $P $V/old/libsdfr.so $V/hnw/libsdfr.so $P $V/old/libsdfr.so $V/hnw/libsdfr.so > gpurun_out/hst.txt 2>&1 || exit 1
cat gpurun_out/hst.txt
REPS=10 timeout -k 10 400 python scripts/conv_time.py $P $V/old/libsdfr.so $V/tns/libsdfr.so $V/tnw/libsdfr.so $P > gpurun_out/tst.txt 2>&1 || exit 1
grep -E "libsdfr| T |total" gpurun_out/tst.txt

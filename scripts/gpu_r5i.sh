#!/bin/bash
# round-5 session: packed colour tail parity + A/B (ngp, fc)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_gpu_render.py tests/test_gpu_fc.py > gpurun_out/t_i.txt 2>&1 || { tail -30 gpurun_out/t_i.txt; exit 1; }
tail -3 gpurun_out/t_i.txt
libs=$(ls -d sdface-gan_amd/lib_var/*/libsdfr.so)
REPS=3 timeout -k 10 400 python scripts/field_time.py sdface-gan_amd/lib/libsdfr.so $libs > gpurun_out/var_ngp.txt 2>&1 || exit 1
grep SUMMARY gpurun_out/var_ngp.txt
NET=fc REPS=3 timeout -k 10 400 python scripts/field_time.py sdface-gan_amd/lib/libsdfr.so $libs > gpurun_out/var_fc.txt 2>&1 || exit 1
grep SUMMARY gpurun_out/var_fc.txt

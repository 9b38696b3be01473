#!/bin/bash
# round 5: blur epilogue variants (rows per segment, columns per thread, row group)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_decoder.py -k "epilogue or decoder_fused" > gpurun_out/j_t.txt 2>&1 || { tail -20 gpurun_out/j_t.txt; exit 1; }; tail -1 gpurun_out/j_t.txt
libs=$(ls -d sdface-gan_amd/lib_var/*/libsdfr.so)
timeout -k 10 400 python scripts/epi_time.py sdface-gan_amd/lib/libsdfr.so $libs > gpurun_out/epi_var.txt 2>&1; rc=$?
grep -E "libsdfr|blur|total" gpurun_out/epi_var.txt; exit $rc

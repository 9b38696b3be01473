#!/bin/bash
# GPU session: interleaved field-time of the product lib and the lib_var/* variants
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
libs=$(ls -d sdface-gan_amd/lib_var/*/libsdfr.so 2>/dev/null)
REPS=${REPS:-3} timeout -k 10 900 python scripts/field_time.py sdface-gan_amd/lib/libsdfr.so $libs > gpurun_out/var.txt 2>&1; r=$?
grep SUMMARY gpurun_out/var.txt; exit $r

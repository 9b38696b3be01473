#!/bin/bash
# GPU session: field-time of the lib_var/* variants (+ the product lib with SDFR_FIELD_X2=1)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
libs=$(ls -d sdface-gan_amd/lib_var/*/libsdfr.so)
timeout -k 10 600 python scripts/field_time.py sdface-gan_amd/lib/libsdfr.so $libs > gpurun_out/var.txt 2>&1; r=$?
SDFR_FIELD_X2=1 timeout -k 10 200 python scripts/field_time.py sdface-gan_amd/lib/libsdfr.so >> gpurun_out/var.txt 2>&1
timeout -k 10 600 python scripts/field_time.py $libs sdface-gan_amd/lib/libsdfr.so >> gpurun_out/var.txt 2>&1
cat gpurun_out/var.txt; exit $r

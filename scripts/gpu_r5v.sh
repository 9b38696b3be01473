#!/bin/bash
# round 5: blur columns-per-thread 5 / 6 variants
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
libs=$(ls -d sdface-gan_amd/lib_var/*/libsdfr.so)
timeout -k 10 400 python scripts/epi_time.py sdface-gan_amd/lib/libsdfr.so $libs sdface-gan_amd/lib/libsdfr.so > gpurun_out/epi_v.txt 2>&1; rc=$?
grep -E "libsdfr|blur|total" gpurun_out/epi_v.txt; exit $rc

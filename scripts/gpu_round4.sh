#!/bin/bash
# Round-4 session: GPU tests, bench, kernel trace, FETCH/WRITE traffic, SQ counters.
set -u
bash scripts/gpu_profile.sh || exit $?
bash scripts/prof_counters.sh

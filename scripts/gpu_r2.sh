#!/bin/bash
set -u
bash scripts/gpu_r.sh || exit $?
KERNELS="r" bash scripts/gpu_cnt.sh

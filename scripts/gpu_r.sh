#!/bin/bash
# field_r_kernel: render + mesh parity with it selected, then field-stage A/B vs p
set -u
mkdir -p gpurun_out
export SDFR_FIELD_KERNEL=${KIND:-r}
export SDFR_PARITY_JSON=gpurun_out/parity_${SDFR_FIELD_KERNEL}.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_mesh.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_r.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_r.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
unset SDFR_FIELD_KERNEL
REPS=3 timeout -k 10 300 python scripts/field_time.py sdface-gan_amd/lib/libsdfr.so@p sdface-gan_amd/lib/libsdfr.so@${KIND:-r} > gpurun_out/ft_r.log 2>&1
rc=$?; echo "ft rc=$rc"; tail -3 gpurun_out/ft_r.log
exit $rc

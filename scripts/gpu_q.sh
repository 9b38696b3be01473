#!/bin/bash
# field_q_kernel: render parity tests with it selected, then field-stage A/B vs field_p_kernel
set -u
mkdir -p gpurun_out
export SDFR_FIELD_KERNEL=q
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_q.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
unset SDFR_FIELD_KERNEL
REPS=3 timeout -k 10 300 python scripts/field_time.py sdface-gan_amd/lib/libsdfr.so@p sdface-gan_amd/lib/libsdfr.so@q > gpurun_out/ft_q.log 2>&1
rc=$?; echo "ft rc=$rc"; tail -3 gpurun_out/ft_q.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
R=$(pwd)
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS"
for k in q p; do
  for pass in 1 2; do
    if [ $pass = 1 ]; then PMC=$P1; else PMC=$P2; fi
    SDFR_FIELD_KERNEL=$k timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "field_${k}_kernel" --output-format csv \
        -d "$R/gpurun_out/pmc_${k}$pass" -o "f$pass" -- python3 "$R/scripts/render_only.py" f16x3 > "gpurun_out/pmc_${k}$pass.log" 2>&1
    rc=$?; echo "pmc $k$pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done

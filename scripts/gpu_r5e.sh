#!/bin/bash
# round 5: conv_t ablations + counters
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python scripts/conv_time.py sdface-gan_amd/lib/libsdfr.so sdface-gan_amd/lib_cvar/*/libsdfr.so \
    > gpurun_out/conv_tvar.txt 2>&1; echo "conv_time rc=$?"; grep -E "lib|T " gpurun_out/conv_tvar.txt
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS"
for pass in 1 2; do
  if [ $pass = 1 ]; then PMC=$P1; else PMC=$P2; fi
  timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "conv_t_kernel" --output-format csv \
      -d "$R/gpurun_out/pmc_convt$pass" -o "t$pass" -- python3 "$R/scripts/decoder_only.py" > gpurun_out/pmc_convt$pass.log 2>&1
  rc=$?; echo "pmc convt$pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

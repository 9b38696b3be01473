#!/bin/bash
# encode-kernel counters: list the gfx950 counters once, then SQ passes on render_only
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
P2="GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_BUSY_avr TD_TD_BUSY_sum"
for pass in 1 2; do
  if [ $pass = 1 ]; then PMC=$P1; else PMC=$P2; fi
  timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-include-regex "ngp_encode_kernel" --output-format csv \
      -d "$R/gpurun_out/pmc_enc$pass" -o "e$pass" -- python3 "$R/scripts/render_only.py" f16x3 > "gpurun_out/pmc_enc$pass.log" 2>&1
  echo "pmc enc$pass rc=$?"
done

#!/bin/bash
# round-5 final: SQ counter passes (field kernels of ngp / siren / fc, decoder convs) and
# the FETCH / WRITE traffic passes over the bench; summaries by summarize_counters.py /
# summarize_profiles.py from gpurun_out/r5final
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5final; mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS"
run() {   # name regex cmd...
    local name=$1 rx=$2; shift 2
    timeout -s KILL 150 rocprofv3 --pmc $PMC --kernel-include-regex "$rx" --output-format csv \
        -d "$R/$O/pmc_$name" -o "$name" -- "$@" > "$O/pmc_$name.log" 2>&1
    local rc=$?; echo "$name rc=$rc"; return $rc
}
PMC=$P1 run ngp_sq1 field_r_kernel python3 "$R/scripts/render_only.py" f16x3 ngp &&
PMC=$P2 run ngp_sq2 field_r_kernel python3 "$R/scripts/render_only.py" f16x3 ngp &&
PMC=$P1 run fc_sq1 field_r_kernel python3 "$R/scripts/render_only.py" f16x3 fc &&
PMC=$P2 run fc_sq2 field_r_kernel python3 "$R/scripts/render_only.py" f16x3 fc &&
PMC=$P1 run siren_sq1 field_p_kernel python3 "$R/scripts/render_only.py" f16x3 siren &&
PMC=$P2 run siren_sq2 field_p_kernel python3 "$R/scripts/render_only.py" f16x3 siren &&
PMC=$P1 run conv_sq1 "conv_[htx]_kernel" python3 "$R/scripts/decoder_only.py" &&
PMC=$P2 run conv_sq2 "conv_[htx]_kernel" python3 "$R/scripts/decoder_only.py" || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/prof_fetch" -o fetch \
    -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras > $O/prof_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/prof_write" -o write \
    -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras > $O/prof_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_trace" -o trace \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/prof_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc

#!/bin/bash
# One parameterised GPU session (replaces the per-session gpu_*.sh one-offs):
#
#   gpurun -- 'bash scripts/gpu.sh <out-dir-name> <task> [<task> ...]'
#
# Tasks run in order, each under its own time limit, output in gpurun_out/<out>/;
# the session stops at the first failure (a GPU step that faulted, aborted or hit its
# limit starts nothing further).  Tasks:
#   smoke                     __graft_entry__.smoke()
#   tests[=<pytest -k expr>]  the -m gpu suite (parity record -> <out>/parity.json)
#   bench                     bench.py, default flags (the driver's command)
#   bench_quick               bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras
#   bench_siren | bench_fc    the other renderers (configs[4])
#   bench_b1                  bench.py --batch 1 --steps 100 (eval.py's one face per call)
#   trace | trace_b1          rocprofv3 --kernel-trace --stats of bench_quick / bench_b1
#   counters                  SQ counter passes: field kernels (ngp, fc, siren), decoder convs
#   traffic                   FETCH_SIZE / WRITE_SIZE passes over bench (one pass each)
#   train1 | train2 | train2find | train2fast   scripts/train_bench.py (stage 1 ngp /
#                             stage 2 / stage 2 with MIOpen find / the same in FAST find mode)
#   prof2 | prof2find         scripts/train_prof.py --stage 2 (torch.profiler breakdown)
#   ddp                       scripts/ddp_cost.py (RCCL world-1 DDP cost)
#   mesh                      scripts/bench_mesh.py
#   py=<script>[,<args>]      python scripts/<script> <args, comma-separated>
#   ab=<n>,<lib>,<lib>...     interleaved bench_quick A/B over SDFR_LIB variants, n rounds
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:?usage: gpu.sh <out> <task>...}; shift; mkdir -p "$O"
export TMPDIR=/tmp SDFR_PARITY_JSON=$R/$O/parity.json
BQ="--steps 20 --warmup 5 --no-cpu-baseline --no-extras"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS"

step() {   # name seconds cmd...  (stdout+stderr -> $O/<name>.log)
    local name=$1 secs=$2; shift 2
    local t0=$(date +%s)
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s :: $(tail -1 "$O/$name.log" | cut -c1-220)"
    return $rc
}
pmc() {    # name regex counters cmd...
    local name=$1 rx=$2 ctr=$3; shift 3
    local t0=$(date +%s)
    timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv \
        -d "$R/$O/pmc_$name" -o "$name" -- "$@" > "$O/pmc_$name.log" 2>&1
    local rc=$?; echo "[pmc $name] rc=$rc $(( $(date +%s) - t0 ))s"; return $rc
}

for task in "$@"; do
    case "$task" in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider \
               --timeout 300 --timeout-method thread ;;
    tests=*) step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider \
               --timeout 300 --timeout-method thread -k "${task#tests=}" ;;
    bench) step bench 600 python bench.py ;;
    bench_quick) step bench_quick 400 python bench.py $BQ ;;
    bench_siren) step bench_siren 300 python bench.py --net siren --steps 10 --warmup 3 --no-extras ;;
    bench_fc) step bench_fc 300 python bench.py --net fc --steps 10 --warmup 3 --no-extras ;;
    bench_b1) step bench_b1 300 python bench.py --batch 1 --steps 100 --warmup 10 --no-cpu-baseline ;;
    trace) step trace 400 rocprofv3 --kernel-trace --stats --output-format csv \
               -d "$R/$O/prof_trace" -o trace -- python3 "$R/bench.py" $BQ ;;
    trace_b1) step trace_b1 300 rocprofv3 --kernel-trace --stats --output-format csv \
               -d "$R/$O/prof_b1" -o b1 -- python3 "$R/bench.py" --batch 1 --steps 100 \
               --warmup 10 --no-cpu-baseline --no-extras ;;
    counters)
        PMC_PY="python3 $R/scripts/render_only.py"
        pmc ngp_sq1 field_r_kernel "$P1" $PMC_PY f16x3 ngp &&
        pmc ngp_sq2 field_r_kernel "$P2" $PMC_PY f16x3 ngp &&
        pmc fc_sq1 field_r_kernel "$P1" $PMC_PY f16x3 fc &&
        pmc fc_sq2 field_r_kernel "$P2" $PMC_PY f16x3 fc &&
        pmc siren_sq1 field_p_kernel "$P1" $PMC_PY f16x3 siren &&
        pmc siren_sq2 field_p_kernel "$P2" $PMC_PY f16x3 siren &&
        pmc conv_sq1 "conv_[htx]_kernel" "$P1" python3 "$R/scripts/decoder_only.py" &&
        pmc conv_sq2 "conv_[htx]_kernel" "$P2" python3 "$R/scripts/decoder_only.py" ;;
    traffic)
        step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/prof_fetch" \
            -o fetch -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras &&
        step prof_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/prof_write" \
            -o write -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras ;;
    train1) step train1 400 python scripts/train_bench.py --stage 1 --net ngp ;;
    train2) step train2 400 python scripts/train_bench.py --stage 2 ;;
    train2find) step train2find 600 python scripts/train_bench.py --stage 2 --miopen-find ;;
    train2fast) MIOPEN_FIND_MODE=2 step train2fast 600 python scripts/train_bench.py --stage 2 \
               --miopen-find ;;
    prof2) step prof2 400 python scripts/train_prof.py --stage 2 --steps 4 --out "$O/prof2.txt" ;;
    prof2find) step prof2find 600 python scripts/train_prof.py --stage 2 --steps 4 --miopen-find \
               --out "$O/prof2find.txt" ;;
    ddp) step ddp 600 python scripts/ddp_cost.py --out "$O/ddp_cost.json" ;;
    mesh) step mesh 300 python scripts/bench_mesh.py ;;
    py=*) a=${task#py=}; IFS=, read -r -a args <<< "$a"
          step "py_$(basename "${args[0]}" .py)" 600 python "scripts/${args[0]}" "${args[@]:1}" ;;
    ab=*) IFS=, read -r -a args <<< "${task#ab=}"; n=${args[0]}; libs=("${args[@]:1}")
          for ((k = 0; k < n; k++)); do
              for L in "${libs[@]}"; do
                  SDFR_LIB=$L step "ab_${k}_$(basename "$(dirname "$L")")" 300 python bench.py $BQ || exit 1
              done
          done ;;
    *) echo "unknown task $task"; exit 2 ;;
    esac || exit 1
done

#!/bin/bash
# All GPU tests, then N short bench runs (no CPU baseline / extras)
set -u
mkdir -p gpurun_out
export SDFR_PARITY_JSON=gpurun_out/parity_full.json
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in $(seq 1 ${NBENCH:-2}); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/bench_full_$i.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_full_$i.log').read().strip().splitlines()[-1])
print('bench', round(d['value'],1), 'ms', round(d['ms_per_step'],3), {k: round(v,3) for k, v in d.get('stage_ms_per_step', {}).items()})"
done

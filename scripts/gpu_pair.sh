#!/bin/bash
# GPU session: pair-kernel A/B vs field_x2_kernel, render parity tests, variant timing
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/pair_ab.py ngp 32 10 > gpurun_out/ab_ngp.json 2> gpurun_out/ab_ngp.err; r=$?; echo "ab rc=$r"; tail -3 gpurun_out/ab_ngp.err; [ $r -eq 0 ] || exit $r
python -c "import json; d=json.load(open('gpurun_out/ab_ngp.json')); print(d['field_ms']); print({k:v[1:] for k,v in d['max_abs_diff_x2_vs_pair'].items()})"
timeout -k 10 600 python -u -m pytest tests/test_gpu_render.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_render.log 2>&1; r=$?; echo "pytest rc=$r"; tail -4 gpurun_out/pt_render.log; [ $r -eq 0 ] || exit $r
libs=$(ls -d sdface-gan_amd/lib_var/*/libsdfr.so 2>/dev/null)
[ -n "${SKIPVAR:-}" ] || timeout -k 10 600 python scripts/field_time.py sdface-gan_amd/lib/libsdfr.so $libs sdface-gan_amd/lib/libsdfr.so $libs > gpurun_out/var.txt 2>&1; cat gpurun_out/var.txt
timeout -k 10 300 python scripts/pair_ab.py siren 8 6 > gpurun_out/ab_siren.json 2> gpurun_out/ab_siren.err; r=$?; echo "ab siren rc=$r"
python -c "import json; d=json.load(open('gpurun_out/ab_siren.json')); print(d['field_ms']); print({k:v[1:] for k,v in d['max_abs_diff_x2_vs_pair'].items()})"
exit $r

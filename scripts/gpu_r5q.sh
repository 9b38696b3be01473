#!/bin/bash
# round 5: 32-bit index math in rgb_finish / epi_blur, vector staging in the mapping / style kernels: parity + bench trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r5q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py \
    tests/test_gpu_render.py -k "epilogue or rgb or decoder or generator or upfirdn or mapping or style or prepared" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/tr" -o tr \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/tr.log 2>&1 || exit 1
tail -1 $O/tr.log | cut -c1-160
timeout -k 10 300 python scripts/epi_time.py > $O/epi.txt 2>&1; grep -E "blur|total" $O/epi.txt

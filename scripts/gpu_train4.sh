#!/bin/bash
# Stage-1 training throughput on HEAD (ngp x3, siren on the HIP GEMMs and on rocBLAS x2),
# then a torch.profiler pass of each network's stage-1 step.
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python scripts/train_bench.py --stage 1 --net ngp --steps 8 --warmup 4 > gpurun_out/tb4_ngp_$i.json 2> gpurun_out/tb4_ngp_$i.err || exit $?
  tail -1 gpurun_out/tb4_ngp_$i.json | cut -c1-160
done
for g in f16x3 torch; do for i in 1 2; do
  timeout -k 10 300 python scripts/train_bench.py --stage 1 --net siren --train-gemm $g --steps 6 --warmup 3 > gpurun_out/tb4_siren_${g}_$i.json 2> gpurun_out/tb4_siren_${g}_$i.err || exit $?
  tail -1 gpurun_out/tb4_siren_${g}_$i.json | cut -c1-160
done; done
timeout -k 10 300 python scripts/train_prof.py --net ngp --out gpurun_out/train4_prof_ngp.txt > /dev/null 2>&1; echo "prof ngp rc=$?"
timeout -k 10 300 python scripts/train_prof.py --net siren --out gpurun_out/train4_prof_siren.txt > /dev/null 2>&1; echo "prof siren rc=$?"

#!/bin/bash
# round 5: non-temporal epilogue stores (conv / blur): A/B by whole bench steps
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
V=sdface-gan_amd/lib_var; P=$R/sdface-gan_amd/lib/libsdfr.so
: > gpurun_out/ntab.txt
for rep in 1 2; do
  for lib in $P $R/$V/nt/libsdfr.so $R/$V/bnt/libsdfr.so; do
    SDFR_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/ntb.log 2>&1 || { tail -5 gpurun_out/ntb.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/ntb.log') if l.startswith('{')][-1])
s=d.get('stage_ms_per_step',{}); print(sys.argv[1][-30:], round(d['value'],1), round(d['ms_per_step'],3), {k:round(v,3) for k,v in s.items()})" $lib >> gpurun_out/ntab.txt
  done
done
cat gpurun_out/ntab.txt

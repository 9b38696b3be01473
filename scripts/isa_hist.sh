#!/bin/bash
# Static instruction histogram of one kernel of field_f16x3.hip (profiling aid).
#   scripts/isa_hist.sh [kernel-symbol-substring] [extra hipcc flags]
set -e
SYM=${1:-field_x_kernelILi0ENS_6NgpNet}
D=$(mktemp -d)
cd "$(dirname "$0")/../sdface-gan_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
    ${2:-} --cuda-device-only -S csrc/field_f16x3.hip -o "$D/k.s"
python3 - "$D/k.s" "$SYM" <<'PY'
import collections, sys
s = open(sys.argv[1]).read()
i = s.index(sys.argv[2]); i = s.index(':\n', i)
body = s[i:s.index('.Lfunc_end', i)].splitlines()
c = collections.Counter(l.split()[0] for l in (x.strip() for x in body)
                        if l and not l.startswith(('.', ';')) and not l.endswith(':'))
print('total', sum(c.values()), ' valu', sum(n for o, n in c.items() if o.startswith('v_') and not o.startswith('v_mfma')))
for op, n in c.most_common(40): print(f'{n:6d} {op}')
PY
rm -rf "$D"

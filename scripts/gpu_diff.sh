set -u
for k in p r; do echo "== $k"; SDFR_FIELD_KERNEL=$k timeout -k 10 120 python scripts/field_diff.py 2>&1 | grep -v amdgpu.ids || exit 1; done

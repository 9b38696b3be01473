"""Print the top kernels of a rocprofv3 --stats run: python scripts/top_kernels.py [dir] [steps]"""
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_t")
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
rows = list(csv.DictReader(open(next(d.glob("*kernel_stats.csv")))))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:18]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:8.3f} ms/step {int(r['Calls']) / steps:5.1f} "
          f"calls {float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:80]}")
print(f"total {tot / steps / 1e6:.3f} ms/step")

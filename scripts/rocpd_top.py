"""Per-kernel totals from a rocprofv3 rocpd database (the default output format):
    python scripts/rocpd_top.py gpurun_out/<dir>/<name>_results.db [N]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
q = ("select s.kernel_name, count(*), avg(d.end - d.start) / 1e6, sum(d.end - d.start) / 1e6 "
     "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
     "group by s.kernel_name order by 4 desc limit ?")
print(f"{'calls':>6} {'avg ms':>9} {'total ms':>9}  kernel")
for name, calls, avg, tot in db.execute(q, (n,)):
    print(f"{calls:6d} {avg:9.3f} {tot:9.2f}  {name[:120]}")

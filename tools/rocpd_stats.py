"""Summarise a rocprofv3 rocpd database (development tool): per kernel name + grid, count and average / median
duration in us, and the average gap between consecutive dispatches.  Usage: python tools/rocpd_stats.py DB [filter]"""
import sqlite3
import statistics
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = c.execute("select name, start, end, grid_x, workgroup_x, lds_size, vgpr_count, accum_vgpr_count, sgpr_count "
                 "from kernels order by start").fetchall()
g = defaultdict(list)
for r in rows:
    if flt in r[0]:
        g[(r[0][:110], r[3], r[4], r[5], r[6], r[7], r[8])].append((r[2] - r[1]) / 1e3)
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    print(f"{len(v):6d} avg {sum(v) / len(v):9.3f} med {statistics.median(v):9.3f} us  grid {k[1]} wg {k[2]} "
          f"lds {k[3]} vgpr {k[4]}+{k[5]} sgpr {k[6]}  {k[0]}")

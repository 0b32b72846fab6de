"""Per-step GPU busy vs. wall and top kernels from a rocprofv3 results.db."""
import sqlite3, sys
from collections import defaultdict
db = sqlite3.connect(sys.argv[1]); cur = db.cursor()
rows = cur.execute("select name, start, end from kernels order by start").fetchall()
# steady state: last 40% of dispatches
rows = rows[int(len(rows) * 0.6):]
busy = sum(e - s for _, s, e in rows); wall = rows[-1][2] - rows[0][1]
gaps = [rows[i + 1][1] - rows[i][2] for i in range(len(rows) - 1)]
print(f"dispatches {len(rows)} busy {busy/1e6:.2f} ms wall {wall/1e6:.2f} ms  idle {100*(1-busy/wall):.1f}%  "
      f"gaps>20us: {sum(g for g in gaps if g > 20000)/1e6:.2f} ms  median gap {sorted(gaps)[len(gaps)//2]/1e3:.1f} us")
agg = defaultdict(float)
for n, s, e in rows: agg[n.split('(')[0].replace('void ugpg::', '').replace('ugpg::', '')[:50]] += e - s
for n, t in sorted(agg.items(), key=lambda x: -x[1])[:16]: print(f"{t/busy*100:5.1f}%  {t/1e6:7.2f} ms  {n}")

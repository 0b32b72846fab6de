"""Per-kernel duration summary of a rocprofv3 --kernel-trace database (rocpd SQLite).

    python tools/kt_summary.py gpurun_out/prof/run_results.db [--match conv3x3] [--top 15]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    q = ("select name, count(*), avg(duration), min(duration), sum(duration) from kernels "
         "where name like ? group by name order by sum(duration) desc limit ?")
    for name, n, avg, mn, tot in c.execute(q, (f"%{a.match}%", a.top)):
        print(f"{n:6d} avg {avg / 1e3:9.2f} us  min {mn / 1e3:9.2f} us  tot {tot / 1e6:8.3f} ms  {name[:110]}")


if __name__ == "__main__":
    main()

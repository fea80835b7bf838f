#!/usr/bin/env python
"""Summarise a rocprofv3 rocpd SQLite database (kernel-trace) as a per-kernel stats table.

    python tools/prof_summary.py gpurun_out/<tag>/prof/prof_results.db [--csv out.csv]

Columns match rocprofv3 --stats (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs).
"""
import sqlite3
import sys


def summary(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     f"from kernels group by {name} order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(r[0], r[1], r[2], r[3], 100.0 * r[2] / tot, r[4], r[5]) for r in rows]


def main():
    db = sys.argv[1]
    rows = summary(db)
    hdr = "Name,Calls,TotalDurationNs,AverageNs,Percentage,MinNs,MaxNs"
    lines = [hdr] + [f'"{n}",{c},{t},{a:.1f},{p:.2f},{mn},{mx}' for n, c, t, a, p, mn, mx in rows]
    if "--csv" in sys.argv:
        open(sys.argv[sys.argv.index("--csv") + 1], "w").write("\n".join(lines) + "\n")
    for n, c, t, a, p, mn, mx in rows:
        print(f"{p:6.2f}%  {c:6d}  avg {a/1e3:9.2f} us  {n[:110]}")


if __name__ == "__main__":
    main()

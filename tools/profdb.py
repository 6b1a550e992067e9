"""Summarise a rocprofv3 SQLite output (`--kernel-trace`, default .db format) per kernel.

    python tools/profdb.py <run_results.db> [steps] [top] [--csv out.csv] [--grid]

Prints ms/step, calls/step and average duration per kernel name (optionally per kernel+grid);
--csv writes the same table in the column layout of rocprofv3's kernel_stats.csv.
"""
import argparse
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("steps", type=float, nargs="?", default=1.0)
    ap.add_argument("top", type=int, nargs="?", default=30)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--grid", action="store_true")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    key = "name || ' grid=' || grid_x || 'x' || grid_y || 'x' || grid_z" if a.grid else "name"
    rows = c.execute(f"select {key}, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     f"from kernels group by {key}").fetchall()
    tot = sum(r[2] for r in rows)
    rows.sort(key=lambda r: -r[2])
    print(f"total {tot / 1e6:.2f} ms  per step {tot / 1e6 / a.steps:.3f} ms")
    for name, n, s, avg, mn, mx in rows[:a.top]:
        print(f"{s / 1e6 / a.steps:7.3f} ms/step {100 * s / tot:5.1f}% n={n / a.steps:6.1f}/step avg={avg / 1e3:8.1f}us "
              f"{name[:110]}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for name, n, s, avg, mn, mx in rows:
                w.writerow([name, n, s, round(avg, 1), round(100 * s / tot, 4), mn, mx])


if __name__ == "__main__":
    main()

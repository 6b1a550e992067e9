"""Per-launch view of one training step from a rocprofv3 kernel-trace .db: every launch of the last
full step (between the last two AdamW kernels) whose name matches a pattern, in launch order, with its
start offset in the step, its stream and duration, and the side-stream kernels it overlapped.

    python tools/launches.py run_results.db <name substring> [--all] [--back N]

--all lists every launch of the step (all kernels), one line each; --back N takes the step N steps
before the last one (default 0: the last full step).
"""
import sqlite3
import sys


def main():
    db, pat = sys.argv[1], sys.argv[2]
    every = "--all" in sys.argv
    back = int(sys.argv[sys.argv.index("--back") + 1]) if "--back" in sys.argv else 0
    c = sqlite3.connect(db)
    rows = c.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    ends = [r[3] for r in rows if r[0].startswith("adamw_kernel")]
    if len(ends) < back + 2:
        print("too few AdamW kernels in the trace")
        return
    t0, t1 = ends[-back - 2], ends[-back - 1]
    win = [r for r in rows if r[2] >= t0 and r[2] < t1]
    print(f"step span {(t1 - t0) / 1e6:.3f} ms, {len(win)} launches")
    for n, s, a, b in win:
        if not every and pat not in n:
            continue
        other = {}
        for n2, s2, a2, b2 in win:
            if s2 == s or b2 <= a or a2 >= b:
                continue
            ov = min(b, b2) - max(a, a2)
            k = n2.split("(")[0][:40]
            other[k] = other.get(k, 0) + ov
        ov = ", ".join(f"{k} {v / 1e3:.0f}us" for k, v in sorted(other.items(), key=lambda x: -x[1])[:3])
        print(f"{(a - t0) / 1e6:8.3f} ms  s{s}  {(b - a) / 1e3:8.1f} us  {n.split('(')[0][:60]:60s} | {ov}")


if __name__ == "__main__":
    main()

"""Per-step GPU timeline from a rocprofv3 kernel-trace .db: busy time of the union of all streams,
per-stream busy time, and idle gaps (no kernel running on any stream) over the last N steps.

    python tools/timeline.py run_results.db [steps] [step_marker_kernel]

The step boundary is the AdamW kernel (one per step).
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    marker = sys.argv[3] if len(sys.argv) > 3 else "adamw_kernel"
    c = sqlite3.connect(db)
    rows = c.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    ends = [r[3] for r in rows if r[0].startswith(marker)]
    if len(ends) < steps + 1:
        steps = len(ends) - 1
    t0, t1 = ends[-steps - 1], ends[-1]
    win = [(s, max(a, t0), min(b, t1)) for n, s, a, b in rows if b > t0 and a < t1]
    busy = 0
    cur_a = cur_b = None
    gaps = []
    for s, a, b in sorted(win, key=lambda x: x[1]):
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
                gaps.append(a - cur_b)
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    busy += cur_b - cur_a
    span = t1 - t0
    per = {}
    for s, a, b in win:
        per[s] = per.get(s, 0) + (b - a)
    print(f"{steps} steps: span {span / steps / 1e6:.3f} ms/step, any-stream busy {busy / steps / 1e6:.3f} ms/step, "
          f"idle {(span - busy) / steps / 1e6:.3f} ms/step in {len(gaps) / steps:.0f} gaps/step")
    for s, v in sorted(per.items()):
        print(f"  stream {s}: kernel time {v / steps / 1e6:.3f} ms/step")


if __name__ == "__main__":
    main()

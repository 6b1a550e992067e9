"""Main-stream kernels of the live step (side stream on) against the same kernels with the side stream off:
per kernel name, ms per step in each trace, the live / serial ratio and the share of the live time that
overlapped side-stream kernels. Last full step of each rocprofv3 kernel-trace .db (between AdamW kernels).

    python tools/live_vs_serial.py live.db serial.db [top]
"""
import collections
import sqlite3
import sys


def step(db, back=1):
    c = sqlite3.connect(db)
    rows = c.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    ends = [r[3] for r in rows if r[0].startswith("adamw_kernel")]
    t0, t1 = ends[-back - 2], ends[-back - 1]
    win = [r for r in rows if t0 <= r[2] < t1]
    main = collections.Counter(r[1] for r in win).most_common(1)[0][0]
    return win, main


def main():
    live, lm = step(sys.argv[1])
    ser, _ = step(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    side = [(a, b) for n, s, a, b in live if s != lm]
    fam = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for n, s, a, b in live:
        if s != lm:
            continue
        k = n.split("(")[0][:70]
        ov = sum(min(b, b2) - max(a, a2) for a2, b2 in side if b2 > a and a2 < b)
        f = fam[k]
        f[0] += b - a
        f[1] += ov
        f[2] += 1
    sfam = collections.Counter()
    for n, s, a, b in ser:
        sfam[n.split("(")[0][:70]] += b - a
    tl = sum(f[0] for f in fam.values())
    ts = sum(sfam[k] for k in fam)
    print(f"main stream live {tl / 1e6:.3f} ms, the same kernels serial {ts / 1e6:.3f} ms "
          f"(+{(tl - ts) / 1e6:.3f}); side-stream kernel time {sum(b - a for a, b in side) / 1e6:.3f} ms")
    rows = sorted(fam.items(), key=lambda x: -(x[1][0] - sfam[x[0]]))
    print(f"{'live ms':>8} {'serial':>7} {'extra':>7} {'ovl':>5} {'n':>3}  kernel (sorted by live - serial)")
    for k, f in rows[:top]:
        s = sfam[k]
        print(f"{f[0] / 1e6:8.3f} {s / 1e6:7.3f} {(f[0] - s) / 1e6:7.3f} {f[1] / max(1, f[0]):5.2f} {f[2]:3d}  {k}")


if __name__ == "__main__":
    main()

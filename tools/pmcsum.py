"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; CSV output).

    python tools/pmcsum.py <fetch counter_collection.csv> <write counter_collection.csv> [kernel substring]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE counts 64 B per 128-B request of a wide coalesced read, so it is doubled; WRITE_SIZE
is exact for 16-B-per-lane stores. Prints MB per dispatch (mean over dispatches) per kernel.
"""
import csv
import gzip
import sys
from collections import defaultdict


def load(path):
    d = defaultdict(list)
    for r in csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)):
        d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return d


def main():
    f, w = load(sys.argv[1]), load(sys.argv[2])
    sub = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = []
    for k in sorted(set(f) | set(w)):
        if sub and sub not in k:
            continue
        fk, wk = f.get(k, [0.0]), w.get(k, [0.0])
        fetch = 2.0 * sum(fk) / len(fk) * 1024 / 1e6
        write = sum(wk) / len(wk) * 1024 / 1e6
        rows.append((fetch + write, fetch, write, len(fk), k))
    rows.sort(reverse=True)
    print(f"{'MB/disp':>9} {'fetchx2':>9} {'write':>9} {'n':>4}  kernel")
    for t, fe, wr, n, k in rows[:40]:
        print(f"{t:9.1f} {fe:9.1f} {wr:9.1f} {n:4d}  {k[:100]}")


if __name__ == "__main__":
    main()

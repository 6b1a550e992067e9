"""Write profiles/pmc_traffic.json from two rocprofv3 --pmc CSV passes of bench.py.

    python tools/pmc_traffic.py <config> <fetch.csv> <write.csv> <label>=<kernel substring> ...

bytes_per_launch = mean over the kernel's dispatches of FETCH_SIZE x 2 + WRITE_SIZE (KiB -> bytes;
FETCH_SIZE doubled: gfx950 counts 64 B per 128-B request of a wide coalesced read,
MI355X_MICROARCH.md 'HBM'). The bench run must launch only that label with this kernel name, or
the substring must be unique to it.
"""
import csv
import json
import os
import sys
from collections import defaultdict


def load(path):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return d


def main():
    config, fpath, wpath = sys.argv[1:4]
    f, w = load(fpath), load(wpath)
    out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    if "ffn0" in data:  # migrate the round-1 flat layout
        data = {"c1": data}
    for spec in sys.argv[4:]:
        label, sub = spec.split("=", 1)
        names = [k for k in f if sub in k]
        if len(names) != 1:
            raise SystemExit(f"{label}: {len(names)} kernels match {sub!r}: {names}")
        k = names[0]
        b = 2 * sum(f[k]) / len(f[k]) * 1024 + sum(w[k]) / len(w[k]) * 1024
        data.setdefault(config, {})[label] = {"kernel": k, "bytes_per_launch": round(b),
                                              "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py "
                                                        f"--config {config}, FETCH_SIZE x2 (gfx950)"}
        print(config, label, k, round(b))
    json.dump(data, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()

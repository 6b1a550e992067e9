"""Write profiles/pmc_traffic.json from two rocprofv3 --pmc CSV passes of bench.py.

    python tools/pmc_traffic.py <config> <fetch.csv> <write.csv> <label>=<spec> ...

<spec> = <kernel substring> (must match exactly one kernel name), or a launch family
"<sub1>|<sub2>...[+<extra sub>]": every kernel matching one of the alternatives counts as a launch
of the family and the dispatches matching <extra sub> add their bytes without counting as launches
(the weight-gradient family: `*_dw=false, false, true|+slab_reduce` charges the split-K slab
reductions to the dW GEMMs whose partial sums they reduce).

bytes_per_launch = (sum over the family's dispatches of FETCH_SIZE x 2 + WRITE_SIZE, KiB -> bytes)
/ number of launch dispatches. FETCH_SIZE doubled: gfx950 counts 64 B per 128-B request of a wide
coalesced read (MI355X_MICROARCH.md 'HBM').
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
        main_spec, _, extra = sub.partition("+")
        alts = [a for a in main_spec.split("|") if a]
        names = [k for k in f if any(a in k for a in alts)]
        if not names or (len(alts) == 1 and not extra and "|" not in main_spec and len(names) != 1):
            raise SystemExit(f"{label}: {len(names)} kernels match {sub!r}: {names}")
        extras = [k for k in f if extra and extra in k] if extra else []
        launches = sum(len(f[k]) for k in names)
        tot = sum(2 * sum(f[k]) * 1024 + sum(w[k]) * 1024 for k in names + extras)
        b = tot / launches
        k = names[0] if len(names) == 1 and not extras else " | ".join(names + [f"+ {e}" for e in extras])
        data.setdefault(config, {})[label] = {"kernel": k, "bytes_per_launch": round(b), "launches": launches,
                                              "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py "
                                                        f"--config {config}, FETCH_SIZE x2 (gfx950)"}
        print(config, label, k, round(b))
    json.dump(data, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()

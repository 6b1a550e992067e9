"""Write profiles/pmc_traffic.json from two rocprofv3 --pmc CSV passes of bench.py.

    python tools/pmc_traffic.py <config> <fetch.csv> <write.csv> <label>=<spec> ...

<spec> = <kernel substring> (must match exactly one kernel name), optionally "@r/m": only the
dispatches whose per-kernel index (dispatch order) is r mod m — the self- and cross-attention
launches of one layer share a kernel and alternate (forward: self first, backward: cross first),
so "attn_fwd_kernel<64@0/2" is the self-attention row and "@1/2" the cross-attention one (applied
per kernel of a family and to its extras too); or a launch family
"<sub1>|<sub2>...[+<extra sub>]": every kernel matching one of the alternatives counts as a launch
of the family and the dispatches matching <extra sub> add their bytes without counting as launches
(the weight-gradient family: `*_dw=false, false, true|+slab_reduce` charges the split-K slab
reductions to the dW GEMMs whose partial sums they reduce).

bytes_per_launch = (sum over the family's dispatches of FETCH_SIZE x 2 + WRITE_SIZE, KiB -> bytes)
/ number of launch dispatches. FETCH_SIZE doubled: gfx950 counts 64 B per 128-B request of a wide
coalesced read (MI355X_MICROARCH.md 'HBM').
"""
import csv
import gzip
import json
import os
import sys
from collections import defaultdict


def load(path):
    rows = defaultdict(list)
    for r in csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)):
        rows[r["Kernel_Name"]].append((int(r.get("Dispatch_Id") or 0), float(r["Counter_Value"])))
    return {k: [v for _, v in sorted(x)] for k, x in rows.items()}


def select(vals, sel):
    if not sel:
        return vals
    r, m = (int(t) for t in sel.split("/"))
    return [v for i, v in enumerate(vals) if i % m == r]


def main():
    config, fpath, wpath = sys.argv[1:4]
    f, w = load(fpath), load(wpath)
    out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    if "ffn0" in data:  # migrate the round-1 flat layout
        data = {"c1": data}
    for spec in sys.argv[4:]:
        label, sub = spec.split("=", 1)
        sub, _, sel = sub.partition("@")
        main_spec, _, extra = sub.partition("+")
        alts = [a for a in main_spec.split("|") if a]
        names = [k for k in f if any(a in k for a in alts)]
        if not names or (len(alts) == 1 and not extra and "|" not in main_spec and len(names) != 1):
            raise SystemExit(f"{label}: {len(names)} kernels match {sub!r}: {names}")
        extras = [k for k in f if extra and extra in k] if extra else []
        launches = sum(len(select(f[k], sel)) for k in names)
        tot = sum(2 * sum(select(f[k], sel)) * 1024 + sum(select(w[k], sel)) * 1024 for k in names + extras)
        if not launches:
            raise SystemExit(f"{label}: no dispatches selected")
        b = tot / launches
        k = names[0] if len(names) == 1 and not extras else " | ".join(names + [f"+ {e}" for e in extras])
        if sel:
            k += f" (dispatches {sel.replace('/', ' mod ')})"
        data.setdefault(config, {})[label] = {"kernel": k, "bytes_per_launch": round(b), "launches": launches,
                                              "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py "
                                                        f"--config {config}, FETCH_SIZE x2 (gfx950)"}
        print(config, label, k, round(b))
    json.dump(data, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()

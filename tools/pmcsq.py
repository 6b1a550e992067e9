"""Per-kernel SQ counter summary from rocprofv3 --pmc CSV passes (sums over dispatches).

    python tools/pmcsq.py <counter_collection.csv> [...]

Prints, per kernel (top by SQ_WAVE_CYCLES): wave-cycle shares of WAIT_ANY (parked at
s_waitcnt/barrier), WAIT_INST_ANY (issue stalls), ACTIVE_INST_ANY; MFMA busy per busy cycle;
LDS bank-conflict share; instruction counts per wave.
"""
import csv
import gzip
import sys
from collections import defaultdict


def main():
    d = defaultdict(lambda: defaultdict(float))
    n = defaultdict(int)
    for path in sys.argv[1:]:
        for r in csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)):
            k = r["Kernel_Name"][:70]
            d[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] in ("SQ_WAVE_CYCLES", "SQ_INSTS_VALU"):
                n[(k, r["Counter_Name"])] += 1
    rows = sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
    print(f"{'kernel':70s} {'wait':>5s} {'stall':>5s} {'activ':>5s} {'mfma%':>6s} {'valu%':>6s} {'lds%':>5s} {'bconf':>6s} {'valu/mfma':>9s}")
    for k, c in rows[:30]:
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        busy = c.get("SQ_BUSY_CYCLES", 0) or 1
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        gui = c.get("GRBM_GUI_ACTIVE", 0) or 1
        print(f"{k:70s} {c.get('SQ_WAIT_ANY',0)/wc:5.2f} {c.get('SQ_WAIT_INST_ANY',0)/wc:5.2f} "
              f"{c.get('SQ_ACTIVE_INST_ANY',0)/wc:5.2f} {mf/(gui*256/8*4) if gui>1 else 0:6.3f} "
              f"{c.get('SQ_ACTIVE_INST_VALU',0)/wc:6.2f} {c.get('SQ_ACTIVE_INST_LDS',0)/wc:5.2f} "
              f"{c.get('SQ_LDS_BANK_CONFLICT',0)/max(1,c.get('SQ_LDS_IDX_ACTIVE',0)):6.2f} "
              f"{c.get('SQ_INSTS_VALU',0)/max(1,c.get('SQ_INSTS_MFMA',0)):9.1f}")


if __name__ == "__main__":
    main()

"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin) per kernel, one line each."""
import re
import sys

cur, rows = None, {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s*(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
keys = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("VGPRs Spill", "vspill"), ("SGPRs Spill", "sspill"),
        ("Occupancy [waves/SIMD]", "occ"), ("LDS Size [bytes/block]", "lds")]
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for name, d in rows.items():
    if flt in name:
        print(f"{name[:60]:60s} " + " ".join(f"{k2}={d.get(k1, '-')}" for k1, k2 in keys))

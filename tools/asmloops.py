"""Inner loops of kernels in a hipcc -S output: instruction mix per loop body (static).

    python tools/asmloops.py file.s <kernel-substring> [...]
"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
for f in re.split(r"\n(?=_Z\w+:)", s):
    name = f.split(":", 1)[0]
    if not any(k in name for k in sys.argv[2:]):
        continue
    lines = f.split("\n")
    labels = {m.group(1): i for i, l in enumerate(lines) for m in [re.match(r"^(\.LBB\w+):", l)] if m}
    print(name[:60])
    for i, l in enumerate(lines):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
        if not m:
            continue
        t = m.group(1) or m.group(2)
        if t not in labels or labels[t] >= i:
            continue
        body = [x.strip() for x in lines[labels[t]:i] if x.startswith("\t") and not x.strip().startswith((".", ";"))]
        c = collections.Counter(x.split()[0] for x in body)
        mf = sum(v for k, v in c.items() if k.startswith("v_mfma"))
        if mf == 0 or len(body) > 1000:
            continue
        valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
        print(f"  loop {t} len={len(body)} mfma={mf} valu={valu} accmov={c['v_accvgpr_mov_b32']} "
              f"accrd={c['v_accvgpr_read_b32']} accwr={c['v_accvgpr_write_b32']} exp={c['v_exp_f32_e32']} "
              f"ds={sum(v for k, v in c.items() if k.startswith('ds_'))} "
              f"scratch={sum(v for k, v in c.items() if k.startswith('scratch'))}")

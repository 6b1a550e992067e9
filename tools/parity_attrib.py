"""Attribute the HIP path's gradient error at a scale fixture.

For a scale fixture (default f_c1: C1 dims, 6 layers) it computes, on the same parameters and batch:
  ref   the fp32 oracle (pinned to the reference's own outputs by tests/test_oracle.py);
  emu   the oracle with every matrix product's operands rounded to bf16 (fp32 accumulation): the
        error floor of a bf16-MFMA implementation of the reference algorithm;
  gpu   the HIP path (when a GPU is present),
and prints the whole-gradient rel-L2 of gpu and emu against ref, the fixture's sampled-entry
metric for both, and per-tensor-group errors (layer x component), so a site whose error exceeds
the bf16 floor stands out.

    python tools/parity_attrib.py [fixture] [--cpu-only]
    python tools/parity_attrib.py [fixture] --sites     (CPU: which rounding sites make the floor)
"""
import os
import re
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "trade-aid-multimodal-transformer_amd"), os.path.join(REPO, "oracle"),
          os.path.join(REPO, "tests"), REPO):
    sys.path.insert(0, p)

import torch  # noqa: E402

import mmt_oracle as O  # noqa: E402
from golden_io import scale_fixture  # noqa: E402


def group_of(k):
    m = re.match(r"blocks\.(\d+)\.(\w+?)\.(\d+)\.(.*)", k)
    if not m:
        return k.split(".")[0] + "." + k.split(".")[1]
    l, kind, _, rest = m.groups()
    part = re.sub(r"heads\.\d+\.", "", rest)
    part = re.sub(r"kv_projections\.\d+\.", "kv.", part)
    return f"L{l}.{kind}.{part}"


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    name = args[0] if args else "f_c1"
    cpu_only = "--cpu-only" in sys.argv or not torch.cuda.is_available()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    z, meta, cfg, sd, idx, tgt = scale_fixture(name)
    t0 = time.time()
    _, r_losses, r_g = O.forward_backward(sd, cfg, idx, tgt)
    t1 = time.time()
    _, e_losses, e_g = O.forward_backward(sd, cfg, idx, tgt, emulate_bf16=True)
    t2 = time.time()
    print(f"{name}: oracle fp32 {t1 - t0:.1f} s, bf16-emulated {t2 - t1:.1f} s")
    names = [k for k in meta["grad_names"]]
    got = {}
    if not cpu_only:
        from test_gpu_scale import build
        m = build(meta, sd)
        m.train()
        logits, losses = m([t.cuda() for t in idx], [t.cuda() for t in tgt])
        sum(losses).backward()
        torch.cuda.synchronize()
        got = {k: g.detach().cpu() for k, g in m.reference_grad_views() if g is not None}
        print("losses gpu", [round(float(l), 6) for l in losses], "ref", [round(float(l), 6) for l in r_losses])
    flat = {"ref": torch.cat([r_g[k].flatten() for k in names]), "emu": torch.cat([e_g[k].flatten() for k in names])}
    if got:
        flat["gpu"] = torch.cat([got[k].flatten() for k in names])
    pick = torch.from_numpy(z["sample_index"])
    print(f"whole-gradient rel-L2 vs fp32 oracle: emu {rel(flat['emu'], flat['ref']):.4f}"
          + (f"  gpu {rel(flat['gpu'], flat['ref']):.4f}  gpu-vs-emu {rel(flat['gpu'], flat['emu']):.4f}" if got else ""))
    print(f"sampled-entry rel-L2 (fixture metric): emu {rel(flat['emu'][pick], flat['ref'][pick]):.4f}"
          + (f"  gpu {rel(flat['gpu'][pick], flat['ref'][pick]):.4f}" if got else ""))
    groups = {}
    for k in names:
        groups.setdefault(group_of(k), []).append(k)
    rows = []
    for gname, ks in groups.items():
        r = torch.cat([r_g[k].flatten() for k in ks])
        e = rel(torch.cat([e_g[k].flatten() for k in ks]), r)
        g = rel(torch.cat([got[k].flatten() for k in ks]), r) if got else float("nan")
        rows.append((gname, r.norm().item(), e, g))
    rows.sort(key=lambda t: -(t[3] if got else t[2]))
    print(f"{'group':48s} {'|ref|':>10s} {'emu':>8s} {'gpu':>8s} {'gpu/emu':>8s}")
    for gname, nrm, e, g in rows:
        print(f"{gname:48s} {nrm:10.3e} {e:8.4f} {g:8.4f} {g / max(e, 1e-12):8.2f}")


def sites(name):
    """Which rounding sites make the bf16 floor: forward-only vs backward-only operand rounding, and
    forward rounding (straight-through) of one GEMM kind at a time."""
    z, meta, cfg, sd, idx, tgt = scale_fixture(name)
    names = meta["grad_names"]
    _, _, rg = O.forward_backward(sd, cfg, idx, tgt)
    ref = torch.cat([rg[k].flatten() for k in names])
    bf, ident = O._bf, (lambda x: x)

    def run_mm(fwd, bwd_saved, bwd_grad):
        class MM(torch.autograd.Function):
            @staticmethod
            def forward(ctx, a, b):
                ctx.save_for_backward(bwd_saved(a), bwd_saved(b))
                return fwd(a) @ fwd(b)

            @staticmethod
            def backward(ctx, g):
                ab, bb = ctx.saved_tensors
                gb = bwd_grad(g)
                ga = gb @ bb.transpose(-2, -1)
                gw = ab.reshape(-1, ab.shape[-1]).t() @ gb.reshape(-1, gb.shape[-1]) if bb.dim() == 2 else ab.transpose(-2, -1) @ gb
                return ga, gw
        old = O._MMBf16
        O._MMBf16 = MM
        try:
            _, _, eg = O.forward_backward(sd, cfg, idx, tgt, emulate_bf16=True)
        finally:
            O._MMBf16 = old
        return rel(torch.cat([eg[k].flatten() for k in names]), ref)

    print(f"{name}: rounding sites -> whole-gradient rel-L2 vs fp32")
    print(f"  all (forward + backward operands)    {run_mm(bf, bf, bf):.4f}")
    print(f"  forward operands only                {run_mm(bf, ident, ident):.4f}")
    print(f"  backward operands only               {run_mm(ident, bf, bf):.4f}")
    print(f"  backward dY only                     {run_mm(ident, ident, bf):.4f}")

    def kind(k):
        if "heads" in k and re.search(r"\.(key|query|value)\.0\.", k):
            return "qkv stage 1"
        if "heads" in k and re.search(r"\.(key|query|value)\.2\.", k):
            return "qkv stage 2"
        for pat, nm in (("sa_layers", "sa proj"), ("net.0", "ffn0"), ("net.2", "ffn2"), ("cross", "cross-attn"),
                        ("post", "output head")):
            if pat in k:
                return nm
        return "other"
    st = lambda x: x.detach().to(torch.bfloat16).float() + (x - x.detach())  # noqa: E731 (forward-only rounding)
    orig = O._lin
    for which in ["qkv stage 1", "qkv stage 2", "sa proj", "ffn0", "ffn2", "cross-attn", "output head"]:
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in sd.items()}
        ids = {id(v): k for k, v in leaves.items()}

        def _lin(x, w, b=None):
            on = kind(ids.get(id(w), "")) == which
            y = (st(x) @ st(w).t()) if on else x @ w.t()
            return y + b if b is not None else y
        O._lin = _lin
        try:
            _, ls = O.forward(leaves, cfg, idx, tgt)
            sum(ls).backward()
        finally:
            O._lin = orig
        e = rel(torch.cat([leaves[k].grad.flatten() for k in names]), ref)
        print(f"  forward rounding of {which:12s} only   {e:.4f}")


if __name__ == "__main__":
    if "--sites" in sys.argv:
        sites(([a for a in sys.argv[1:] if not a.startswith("--")] or ["f_c1"])[0])
    else:
        main()

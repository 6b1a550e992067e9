"""Fused AdamW on the gfx950 library — drop-in for torch.optim.AdamW(m.parameters(), lr=...)
(reference main.py:464, 648-650).

Semantics follow torch's AdamW defaults: betas (0.9, 0.999), eps 1e-8, weight_decay 0.01,
decoupled decay, bias correction; parameters whose .grad is None are skipped entirely (the
model's `flat_unused`, the CrossAttention parameters that never get a gradient). The stock
torch.optim.AdamW gives the same result on the model (tests/test_gpu_model.py); this one runs the
update as one fused HIP kernel over the flat buffer.
"""
import torch

import mmt_lib as ML


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = ML.lib()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.device.type != "cuda" or p.dtype != torch.float32:
                    raise RuntimeError("mmt AdamW runs on fp32 ROCm tensors only (no CPU path)")
                g = p.grad
                if not g.is_contiguous() or not p.is_contiguous():
                    raise RuntimeError("mmt AdamW needs contiguous params/grads")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                n = p.numel()
                rc = L.mmt_adamw_step(None, ML.stream_ptr(p.device), ML.ptr(p), ML.ptr(g), ML.ptr(st["exp_avg"]),
                                      ML.ptr(st["exp_avg_sq"]), n, st["step"], group["lr"], b1, b2, group["eps"],
                                      group["weight_decay"])
                ML.check(rc, None, "mmt_adamw_step")
        return loss

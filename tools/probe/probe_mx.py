"""Dev probe: run tools/probe/probe_mx.hip on the GPU and print what the scaled fp8 MFMA and the fp8
pack conversion do (k layout, scale bytes, encoding). Build: hipcc -shared -fPIC --offload-arch=gfx950."""
import ctypes
import os
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe_mx.so"))
torch.manual_seed(0)
# exactly representable e4m3 values
vals = torch.tensor([-2.0, -1.5, -1.0, -0.5, 0.0, 0.5, 1.0, 1.5, 2.0])
A = vals[torch.randint(0, 9, (32, 64))]
B = vals[torch.randint(0, 9, (64, 32))]
def lanes(M, rowmajor):  # lane l: row/col l&31, k = 32*(l>>5) + j
    out = torch.empty(64, 32)
    for l in range(64):
        r, h = l & 31, l >> 5
        out[l] = M[r, 32 * h:32 * h + 32] if rowmajor else M[32 * h:32 * h + 32, r]
    return out.to(torch.float8_e4m3fn).view(torch.uint8).contiguous()
a = lanes(A, True).cuda()
b = lanes(B, False).cuda()
def run(sa, sb):
    d = torch.zeros(64, 16, device="cuda")
    assert L.probe_mx(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(sa.data_ptr()),
                      ctypes.c_void_p(sb.data_ptr()), ctypes.c_void_p(d.data_ptr())) == 0
    D = torch.empty(32, 32)
    dc = d.cpu()
    for l in range(64):
        for reg in range(16):
            D[(reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5), l & 31] = dc[l, reg]
    return D
one = torch.full((64,), 127, dtype=torch.int32, device="cuda")
D = run(one, one)
print("unscaled max err", (D - A @ B).abs().max().item())
# scale byte select: bytes 127,128,129,130 -> which applies
sb4 = torch.full((64,), 127 | (128 << 8) | (129 << 16) | (126 << 24), dtype=torch.int32, device="cuda")
D = run(sb4, one)
print("multi-byte scale ratio", (D / (A @ B)).nanmean().item())
# per-lane-half scale: lanes 32..63 (k block 1) scaled by 2
sh = torch.tensor([127] * 32 + [128] * 32, dtype=torch.int32, device="cuda")
D = run(sh, one)
ref = A[:, :32] @ B[:32] + 2 * (A[:, 32:] @ B[32:])
print("half-lane scale err", (D - ref).abs().max().item())
# per-row scale: lane l&31 = row r scaled by 2^(r%3)
sr = torch.tensor([127 + (l & 31) % 3 for l in range(64)], dtype=torch.int32, device="cuda")
D = run(sr, one)
ref = torch.diag(torch.tensor([2.0 ** (r % 3) for r in range(32)])) @ (A @ B)
print("per-row scale err", (D - ref).abs().max().item())
# conversion: random floats vs torch's e4m3fn rounding
x = torch.randn(4096) * 50
y = torch.zeros(1024, dtype=torch.int32, device="cuda")
xd = x.cuda()
assert L.probe_cvt(ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(y.data_ptr()), 1024) == 0
got = y.cpu().view(torch.uint8)
ref = x.to(torch.float8_e4m3fn).view(torch.uint8)
print("cvt mismatches", int((got != ref).sum()), "of", got.numel())
big = torch.tensor([500.0, -1000.0, 448.0, 1e-9] * 4)
y2 = torch.zeros(4, dtype=torch.int32, device="cuda")
assert L.probe_cvt(ctypes.c_void_p(big.cuda().data_ptr()), ctypes.c_void_p(y2.data_ptr()), 4) == 0
print("saturation bytes", [hex(v) for v in y2.cpu().view(torch.uint8)[:4].tolist()],
      "torch", [hex(v) for v in big[:4].to(torch.float8_e4m3fn).view(torch.uint8).tolist()])
# which (lane half, byte) -> K-block mapping do the scales follow? candidates: the scale of lane
# r + 32*b applies to "block b" = a set of my-layout k indices
D = run(sh, one)
cands = {
    "k=32h+j, block=h": [list(range(0, 32)), list(range(32, 64))],
    "block0={h0 j<16, h1 j<16}": [list(range(0, 16)) + list(range(32, 48)), list(range(16, 32)) + list(range(48, 64))],
    "block0=even 8-groups": [[k for k in range(64) if (k // 8) % 2 == 0], [k for k in range(64) if (k // 8) % 2 == 1]],
    "block0=even 4-groups": [[k for k in range(64) if (k // 4) % 2 == 0], [k for k in range(64) if (k // 4) % 2 == 1]],
}
for name, (b0, b1) in cands.items():
    ref = A[:, b0] @ B[b0] + 2 * (A[:, b1] @ B[b1])
    print("cand", name, (D - ref).abs().max().item())
# scale of B per column
D = run(one, sh)
for name, (b0, b1) in cands.items():
    ref = A[:, b0] @ B[b0] + 2 * (A[:, b1] @ B[b1])
    print("candB", name, (D - ref).abs().max().item())

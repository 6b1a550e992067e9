import ctypes, os, torch
here = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(here, "libprobe_tr.so"))
rows = torch.zeros(64, dtype=torch.int32); cols = torch.zeros(64, dtype=torch.int32)
for l in range(64):
    g, i = l >> 4, l & 15
    q, p = i >> 2, i & 3
    rows[l] = 4 * (g >> 1) + q          # group pairs read rows 0-3 / 4-7
    cols[l] = 16 * (g & 1) + 4 * p
r, c = rows.cuda(), cols.cuda()
out = torch.zeros(64 * 4, dtype=torch.int16, device="cuda")
L.probe_tr(ctypes.c_void_p(r.data_ptr()), ctypes.c_void_p(c.data_ptr()), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
o = out.cpu().view(64, 4)
for l in range(64):
    vals = o[l].tolist()
    print(l, [(v // 64, v % 64) for v in vals])

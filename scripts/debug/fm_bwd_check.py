"""Compare the F2 partial sums (Z = G^T X rows 0..16, t = (x^2)^T g) with torch."""
import sys
import torch
sys.path.insert(0, ".")
from dmlc_core_amd import _dmlc

torch.manual_seed(0)
for dim, rows in ((128, 37), (128, 64), (256, 32)):
    x8 = (torch.randn(rows, dim, device="cuda") * 2).to(torch.float8_e4m3fn)
    g = torch.randn(rows, device="cuda")
    xv = torch.randn(rows, 16, device="cuda")
    nblk = 2
    part = torch.empty((nblk, 18, dim), device="cuda")
    _dmlc.fm_backward(x8.data_ptr(), rows, dim, g.data_ptr(), xv.data_ptr(), nblk, part.data_ptr(),
                      int(torch.cuda.current_stream().cuda_stream))
    z = part.sum(0)
    x = x8.float()
    G = torch.cat([g[:, None], g[:, None] * xv], 1).bfloat16().float()
    Z = G.t() @ x
    t = (x * x).t() @ g
    for c in (0, 1, 5, 16):
        e = (z[c] - Z[c]).abs().max().item() / (Z[c].abs().max().item() + 1e-9)
        print(dim, rows, "Z row", c, "rel err", round(e, 5))
    e = (z[17] - t).abs().max().item() / t.abs().max().item()
    print(dim, rows, "t rel err", round(e, 5))
    # where does Z[0] differ?
    d = (z[0] - Z[0]).abs()
    bad = (d > 1e-3 * Z[0].abs().max()).nonzero().flatten()[:20].tolist()
    print("bad features of Z0:", bad)

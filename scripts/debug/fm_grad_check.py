"""HashedFM autograd (HIP kernels) vs fp32 autograd, per gradient."""
import sys
import torch
sys.path.insert(0, ".")
from dmlc_core_amd.models import HashedFM

for dim, rows in ((128, 37), (512, 1000)):
    torch.manual_seed(dim + rows)
    x8 = (torch.randn(rows, dim, device="cuda") * 2).to(torch.float8_e4m3fn)
    scale = 0.5
    m = HashedFM(dim=dim).cuda()
    with torch.no_grad():
        m.w.normal_(0, 0.05)
        m.v.normal_(0, 0.05)
        m.bias.fill_(0.3)
    r = torch.randn(rows, device="cuda")
    (m(x8, scale) * r).sum().backward()
    x = x8.float() / scale
    w = m.w.detach().clone().requires_grad_(True)
    v = m.v.detach().clone().requires_grad_(True)
    b = m.bias.detach().clone().requires_grad_(True)
    ref = HashedFM.reference(x, w, v, b)
    (ref * r).sum().backward()
    for name, got, want in (("w", m.w.grad, w.grad), ("v", m.v.grad, v.grad), ("b", m.bias.grad, b.grad)):
        err = (got - want).abs().max().item() / (want.abs().max().item() + 1e-6)
        print(dim, rows, name, got.shape, want.shape, "rel err", err)
        if err > 1e-2:
            print(" got", got.flatten()[:6].tolist())
            print(" want", want.flatten()[:6].tolist())

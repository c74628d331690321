"""Three-way check HIP vs oracle-on-CPU vs oracle-on-GPU for test_layer_vs_oracle_larger's setup."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
from oracle import stgcn_oracle as O  # noqa: E402

P = ge.load_package()
DEV = "cuda:0"
cin, cout, stride, norm = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
torch.manual_seed(7)
N, T = 4, 64
A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32)
layer = P.StgcnLayer(cin, cout, (9, 25), 3, 25, stride=stride, normalization=norm)
with torch.no_grad():
    for name, p in layer.named_parameters():
        if "tcn.0" in name or "tcn.3" in name or "residual.1" in name:
            p.add_(0.1 * torch.randn(p.shape))
M = 1 + 0.1 * torch.randn(3, 25, 25)
x = torch.randn(N, cin, T, 25)
dy = torch.randn(N, cout, (T - 1) // stride + 1, 25)


def run_oracle(dev):
    sd = {k: v.clone().to(dev).requires_grad_(True) for k, v in layer.state_dict().items()}
    xr = x.clone().to(dev).requires_grad_(True)
    Ar = (A * M).to(dev).requires_grad_(True)
    ref = O.stgcn_layer(xr, Ar, sd, "", 9, stride, True, norm)
    ref.backward(dy.to(dev))
    return ref.detach().cpu(), xr.grad.cpu(), Ar.grad.cpu(), {k: v.grad.cpu() for k, v in sd.items() if v.grad is not None}


def rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max()).item()


yc, dxc, dAc, gc = run_oracle("cpu")
yg, dxg, dAg, gg = run_oracle(DEV)
lay = layer.to(DEV)
xh = x.to(DEV).requires_grad_(True)
Ah = (A * M).to(DEV).requires_grad_(True)
yh = lay(xh, Ah)
yh.backward(dy.to(DEV))
print("y   hip-cpu %.2e hip-gpu %.2e gpu-cpu %.2e" % (rel(yh.detach().cpu(), yc), rel(yh.detach().cpu(), yg), rel(yg, yc)))
print("dx  hip-cpu %.2e hip-gpu %.2e gpu-cpu %.2e" % (rel(xh.grad.cpu(), dxc), rel(xh.grad.cpu(), dxg), rel(dxg, dxc)))
print("dA  hip-cpu %.2e hip-gpu %.2e gpu-cpu %.2e" % (rel(Ah.grad.cpu(), dAc), rel(Ah.grad.cpu(), dAg), rel(dAg, dAc)))
named = dict(lay.named_parameters())
for k in gc:
    print("%-22s hip-cpu %.2e hip-gpu %.2e gpu-cpu %.2e" % (k, rel(named[k].grad.cpu(), gc[k]), rel(named[k].grad.cpu(), gg[k]), rel(gg[k], gc[k])))
e = (xh.grad.cpu().double() - dxc.double()).abs()
thr = 1e-3 * dxc.abs().max().item()
print("dx: n elems", e.numel(), "n > 1e-3*max:", int((e > thr).sum()), "L2 rel %.2e" % (
    ((xh.grad.cpu().double() - dxc.double()).norm() / dxc.double().norm()).item()))
# near-zero pre-activations at the final relu
pre = yh.detach().cpu()
print("y==0 fraction %.3f, |y|<1e-5 & >0: %d" % ((pre == 0).float().mean().item(), int(((pre > 0) & (pre < 1e-5)).sum())))
print("yc==0 vs yh==0 mismatches:", int(((yc == 0) != (pre == 0)).sum()))

"""Compare every intermediate gradient of the HIP StgcnLayer backward with torch autograd (GPU fp32).
Usage: python tools/debug_layer2.py CIN COUT STRIDE"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

P = ge.load_package()
K = P.native
dev = "cuda:0"
cin, cout, stride = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
torch.manual_seed(7)
N, T, V = 4, 64, 25
A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32, device=dev)
layer = P.StgcnLayer(cin, cout, (9, 25), 3, 25, stride=stride, normalization="BatchNorm").to(dev)
x = torch.randn(N, cin, T, V, device=dev)
sd = dict(layer.named_parameters())


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()


# torch reference with retained intermediates
xr = x.clone().requires_grad_(True)
z = F.conv2d(xr, sd["gcn.conv.weight"], sd["gcn.conv.bias"]).view(N, 3, cout * T, V)
g = torch.matmul(z, A).sum(1).view(N, cout, T, V)
g.retain_grad()
h = torch.relu(F.batch_norm(g, None, None, sd["tcn.0.weight"], sd["tcn.0.bias"], training=True))
h.retain_grad()
u = F.conv2d(h, sd["tcn.2.weight"], sd["tcn.2.bias"], stride=(stride, 1), padding=(4, 0))
u.retain_grad()
b2 = F.batch_norm(u, None, None, sd["tcn.3.weight"], sd["tcn.3.bias"], training=True)
if layer.is_residual_conv:
    r = F.conv2d(xr, sd["residual.0.weight"], sd["residual.0.bias"], stride=(stride, 1))
    res = F.batch_norm(r, None, None, sd["residual.1.weight"], sd["residual.1.bias"], training=True)
else:
    res = xr
y = torch.relu(b2 + res)
dy = torch.randn_like(y)
y.backward(dy)

# HIP path, hooking intermediates by monkeypatching native calls
captured = {}
orig_conv = K.conv_rows


def conv_spy(*a, **k):
    out = orig_conv(*a, **k)
    captured.setdefault("conv", []).append(out)
    return out


K.conv_rows = conv_spy
orig_apply = K.bn_bwd_apply


def apply_spy(dy_, M, C, out, **k):
    r_ = orig_apply(dy_, M, C, out, **k)
    captured.setdefault("apply", []).append(out.clone())
    return r_


K.bn_bwd_apply = apply_spy
orig_trans = K.amix_trans


def trans_spy(dw, A_, Cin, out, accumulate):
    captured["dx_before_amix"] = out.clone()
    captured["DW"] = dw
    r_ = orig_trans(dw, A_, Cin, out, accumulate)
    captured["dx_after"] = out.clone()
    return r_


K.amix_trans = trans_spy
xg = x.clone().requires_grad_(True)
yg = layer(xg, A)
print("y", rel(yg, y))
yg.backward(dy)
convs = captured["conv"]
print("fwd g", rel(convs[0], g), "u", rel(convs[1], u))
print("n conv calls", len(convs), "n apply", len(captured["apply"]))
ap = captured["apply"]
print("du", rel(ap[0], u.grad))
for i, c in enumerate(convs[2:]):
    print("bwd conv", i, tuple(c.shape))
dh = [c for c in convs[2:] if c.shape == h.shape][0]
print("dh", rel(dh, h.grad))
print("dg", rel(ap[-1], g.grad))
print("dx total", rel(xg.grad, xr.grad))

"""Stage-by-stage comparison of the HIP StgcnLayer backward against torch fp32 autograd (GPU).
Usage: python tools/debug_layer.py CIN COUT STRIDE NORM"""
import sys
import os
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

P = ge.load_package()
K = P.native
dev = "cuda:0"
cin, cout, stride, norm = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
torch.manual_seed(7)
N, T, V = 4, 64, 25
A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32, device=dev)
x = torch.randn(N, cin, T, V, device=dev)
Wg = torch.randn(3 * cout, cin, 1, 1, device=dev) / cin ** 0.5
bg = torch.randn(3 * cout, device=dev) * 0.1
# stage 1: GCN
xr = x.clone().requires_grad_(True)
z = F.conv2d(xr, Wg, bg).view(N, 3, cout * T, V)
g_ref = torch.matmul(z, A).sum(1).view(N, cout, T, V)
dg = torch.randn_like(g_ref)
g_ref.backward(dg)
xc = K.to_rows(x, torch.float32)
XA = K.amix_fwd(xc, A)
wg3 = Wg.view(3, cout, cin).permute(1, 0, 2).reshape(1, cout, 3 * cin)
wgp, cp, kp = K.pack_weight(wg3, torch.float32)
bias2d = K.gcn_bias(A, bg, N, cout)
g = K.conv_rows(XA, wgp, 3 * cin, cout, cp, kp, T, T, bias=bias2d, bias_mode=2)
print("g rel err", ((g - g_ref).abs().max() / g_ref.abs().max()).item())
wgT = Wg.view(3, cout, cin).permute(0, 2, 1).reshape(1, 3 * cin, cout)
wgTp, cq, kq = K.pack_weight(wgT, torch.float32)
dgc = K.to_rows(dg, torch.float32)
DW = K.conv_rows(dgc, wgTp, cout, 3 * cin, cq, kq, T, T)
# reference DW: dz = dg @ A^T per p ; DW[w][p,ci] = sum_c dg[w][c] W[p*C+c][ci]
DW_ref = torch.einsum("nctw,pcd->npdtw", dg, Wg.view(3, cout, cin)).reshape(N, 3 * cin, T, V)
print("DW rel err", ((DW - DW_ref).abs().max() / DW_ref.abs().max()).item())
dx = K.cl_empty(N, cin, T, V, torch.float32, dev)
K.amix_trans(DW, A, cin, dx, accumulate=False)
print("dx(gcn) rel err", ((dx - xr.grad).abs().max() / xr.grad.abs().max()).item())
# stage 2: TCN dgrad
Wt = torch.randn(cout, cout, 9, 1, device=dev) / (cout * 9) ** 0.5
h = torch.randn(N, cout, T, V, device=dev).requires_grad_(True)
u = F.conv2d(h, Wt, None, stride=(stride, 1), padding=(4, 0))
du = torch.randn_like(u)
u.backward(du)
wtT = Wt.squeeze(-1).permute(2, 1, 0)
wtTp, cq, kq = K.pack_weight(wtT, torch.float32)
dh = K.conv_rows(K.to_rows(du, torch.float32), wtTp, cout, cout, cq, kq, u.shape[2], T, Kt=9, stride=stride, pad=4,
                 trans=True)
print("dh rel err", ((dh - h.grad).abs().max() / h.grad.abs().max()).item())

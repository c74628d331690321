"""Debug the fused layer kernel: identity temporal weight (z = h) isolates phase 1; report error maps."""
import sys, os
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
from oracle import stgcn_oracle as O
P = ge.load_package(); K = P.native
DEV = "cuda:0"; BF = torch.bfloat16
rb = lambda t: t.to(BF).float()
N, T, V, C = int(sys.argv[1]), int(sys.argv[2]), 25, 64
torch.manual_seed(0)
A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32)
Pp = A.shape[0]
x = rb(torch.randn(N, C, T, V))
wg = rb(torch.randn(Pp * C, C, 1, 1) / C ** 0.5); bg = torch.zeros(Pp * C)
sc, sh = torch.ones(C), torch.zeros(C)
for mode in ("delta", "rand"):
    if mode == "delta":
        wt = torch.zeros(C, C, 9, 1); wt[:, :, 4, 0] = torch.eye(C)
    else:
        wt = rb(torch.randn(C, C, 9, 1) / (9 * C) ** 0.5)
    bt = torch.zeros(C)
    g = O.tgcn(x, wg, bg, A)
    h = torch.relu(g * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
    ref = F.conv2d(rb(h), wt, bt, padding=(4, 0))
    A_d = A.to(DEV)
    bias2d = K.gcn_bias(A_d, bg.to(DEV), N, C)
    wgf = wg.view(Pp, C, C).permute(1, 0, 2).reshape(C, Pp * C).to(DEV)
    wimg, cpg, kwg = K.pack_gcn_weight(wgf, BF)
    wtp, _, _ = K.pack_weight(wt.squeeze(-1).permute(2, 0, 1).to(DEV), BF, stride=1)
    xd = x.to(DEV, BF).contiguous(memory_format=torch.channels_last)
    z = K.layer_fused(xd, A_d, wimg, bias2d, sc.to(DEV), sh.to(DEV), wtp, bt.to(DEV), stats=None)
    torch.cuda.synchronize()
    zf = z.float().cpu()
    err = (zf - ref).abs()
    print(mode, "max err", err.max().item(), "scale", ref.abs().max().item())
    e_t = err.amax(dim=(0, 1, 3)); e_v = err.amax(dim=(0, 1, 2)); e_c = err.amax(dim=(0, 2, 3))
    print(" err by frame", [round(v, 2) for v in e_t.tolist()])
    print(" err by joint", [round(v, 2) for v in e_v.tolist()])
    print(" err by chan", [round(v, 2) for v in e_c.tolist()])
    n0 = (0, slice(None), 5, 3)
    print(" z[0,:8,5,3]", zf[0, :8, 5, 3].tolist()); print(" r[0,:8,5,3]", ref[0, :8, 5, 3].tolist())

"""Debug 2: identity graph conv (A = I, P = 1, W' = I) isolates phase 2; gcn_tile output vs oracle checks the
graph conv on the same data."""
import sys, os
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
from oracle import stgcn_oracle as O
P = ge.load_package(); K = P.native
DEV = "cuda:0"; BF = torch.bfloat16
rb = lambda t: t.to(BF).float()
N, T, V, C = 1, 20, 25, 64
torch.manual_seed(0)
x = rb(torch.randn(N, C, T, V))
xd = x.to(DEV, BF).contiguous(memory_format=torch.channels_last)
sc, sh = torch.ones(C), torch.zeros(C)
bt = torch.zeros(C)
def rep(name, z, ref):
    err = (z - ref).abs()
    print(name, "max err", err.max().item(), "scale", ref.abs().max().item())
    print("  by joint", [round(v, 2) for v in err.amax(dim=(0, 1, 2)).tolist()])
    print("  by frame", [round(v, 2) for v in err.amax(dim=(0, 1, 3)).tolist()])
# identity graph conv
A1 = torch.eye(V).unsqueeze(0)
wg1 = torch.eye(C).view(C, C, 1, 1)
for mode in ("delta", "rand"):
    if mode == "delta":
        wt = torch.zeros(C, C, 9, 1); wt[:, :, 4, 0] = torch.eye(C)
    else:
        wt = rb(torch.randn(C, C, 9, 1) / (9 * C) ** 0.5)
    ref = F.conv2d(rb(torch.relu(x)), wt, bt, padding=(4, 0))
    A_d = A1.to(DEV)
    wimg, cpg, kwg = K.pack_gcn_weight(torch.eye(C).to(DEV), BF)
    wtp, _, _ = K.pack_weight(wt.squeeze(-1).permute(2, 0, 1).to(DEV), BF, stride=1)
    z = K.layer_fused(xd, A_d, wimg, None, sc.to(DEV), sh.to(DEV), wtp, bt.to(DEV), stats=None)
    torch.cuda.synchronize()
    rep("identity-gcn " + mode, z.float().cpu(), ref)
# gcn_tile on the real graph vs oracle
A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32)
Pp = A.shape[0]
wg = rb(torch.randn(Pp * C, C, 1, 1) / C ** 0.5)
g = O.tgcn(x, wg, torch.zeros(Pp * C), A)
A_d = A.to(DEV)
sup = K.GraphSupport(A_d)
wgf = wg.view(Pp, C, C).permute(1, 0, 2).reshape(C, Pp * C).to(DEV)
wimg, cpg, kwg = K.pack_gcn_weight(wgf, BF)
gt = K.gcn_tile(xd, A_d, wimg, kwg, C, C, cpg, sup)
torch.cuda.synchronize()
rep("gcn_tile", gt.float().cpu(), g)
wt = torch.zeros(C, C, 9, 1); wt[:, :, 4, 0] = torch.eye(C)
wtp, _, _ = K.pack_weight(wt.squeeze(-1).permute(2, 0, 1).to(DEV), BF, stride=1)
z = K.layer_fused(xd, A_d, wimg, None, sc.to(DEV), sh.to(DEV), wtp, bt.to(DEV), stats=None)
torch.cuda.synchronize()
rep("fused(delta) vs relu(gcn_tile)", z.float().cpu(), torch.relu(gt.float().cpu()))
rep("fused(delta) vs relu(oracle)", z.float().cpu(), rb(torch.relu(g)))

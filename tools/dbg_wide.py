"""Locate conv_wide errors (C=128, Kt=9, s1) vs torch fp32: which (n, t, v, c) are wrong, per N."""
import sys, os
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
P = ge.load_package(); K = P.native
DEV = "cuda:0"; BF = torch.bfloat16
def cl(x, dt=torch.float32): return x.to(DEV, dt).contiguous(memory_format=torch.channels_last)
rb = lambda t: t.to(BF).float()
C, T, V = int(sys.argv[1]), int(sys.argv[2]), 25
for N in [int(v) for v in sys.argv[3].split(",")]:
    torch.manual_seed(0)
    w = rb(torch.randn(C, C, 9, 1) / (C * 9) ** 0.5)
    for mode in ("fwd_pro0", "trans"):
        x = rb(torch.randn(N, C, T, V))
        if mode == "fwd_pro0":
            ref = F.conv2d(x, w, None, padding=(4, 0))
            wp, cp, kp = K.pack_weight(w.squeeze(-1).permute(2, 0, 1).to(DEV), BF)
            y = K.conv_rows(cl(x, BF), wp, C, C, cp, kp, T, T, Kt=9, pad=4)
        else:
            xr = torch.zeros_like(x).requires_grad_(True)
            F.conv2d(xr, w, None, padding=(4, 0)).backward(x)
            ref = xr.grad
            wp, cp, kp = K.pack_weight(w.squeeze(-1).permute(2, 1, 0).to(DEV), BF, trans=True)
            y = K.conv_rows(cl(x, BF), wp, C, C, cp, kp, T, T, Kt=9, pad=4, trans=True)
        torch.cuda.synchronize()
        e = (y.float().cpu() - ref).abs()
        bad = e > 2e-2 * ref.abs().max()
        print(f"N={N} {mode}: max rel {e.max().item() / ref.abs().max().item():.3e}  bad {int(bad.sum())} / {bad.numel()}",
              flush=True)
        if bad.any():
            idx = bad.nonzero()
            ns = sorted(set(idx[:, 0].tolist())); ts = sorted(set(idx[:, 2].tolist()))
            cs = sorted(set(idx[:, 1].tolist())); vs = sorted(set(idx[:, 3].tolist()))
            print("  n:", ns[:20], len(ns), " t:", ts[:40], len(ts), " c:", cs[:10], len(cs), " v:", vs[:25])

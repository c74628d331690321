"""Cycle accounts of the row-streaming temporal conv (tconv_frame.hip, STGCN_TCR_DBG & 256 build):
STGCN_LIB=<that build> python tools/tcr_prof.py [fwd|dgrad]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

K = ge.load_package().native
dev = "cuda:0"
mode = sys.argv[1] if len(sys.argv) > 1 else "dgrad"
N, T, V, C = 64, 300, 25, 64
x = torch.randn(N, C, T, V, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = torch.randn(9, C, C, device=dev) * 0.05
wp, cp, kp = K.pack_weight(w, torch.bfloat16, stride=1, trans=mode == "dgrad")
sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
for _ in range(20):
    if mode == "dgrad":
        y = K.tconv_frame(x, wp, cp, kp, trans=True)
    else:
        y = K.tconv_frame(x, wp, cp, kp, pro_a=sc, pro_b=sh)
torch.cuda.synchronize()
nb = N * max(1, 256 // N)  # the row form's blocks (rplan: 256 / N runs per sample at these shapes)
raw = y.permute(0, 2, 3, 1).contiguous().view(-1).view(torch.float32)[: nb * 8 * 8].cpu().view(nb, 8, 8)
names = ["kloop", "B1", "ep_write", "B2", "readback", "xform", "total", "nsteps"]
m = raw.mean(dim=(0, 1))
print(mode, " ".join(f"{n}={v:.0f}" for n, v in zip(names, m.tolist())))
print("per step:", " ".join(f"{n}={v / m[7]:.0f}" for n, v in zip(names[:6], m[:6].tolist())))
print("kloop cycles per MFMA (72 per wave per step):", float(m[0] / m[7] / 72))

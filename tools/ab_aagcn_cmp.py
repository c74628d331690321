"""Compare two tools/ab_aagcn.py outputs (new, old): each build's bf16 vs the fp32 run, per tensor."""
import sys

import torch

a = torch.load(sys.argv[1])
b = torch.load(sys.argv[2])


def l2(t, r):
    return ((t - r).norm() / r.norm().clamp_min(1e-300)).item()


f = b["fp32"]
print("fp32 new vs old: logits", l2(a["fp32"]["logits"], f["logits"]), "dx", l2(a["fp32"]["dx"], f["dx"]))
ks = [k for k in f if not k.endswith("tcn.2.bias") and not k.endswith("residual.0.bias") and not k.endswith("phi.bias")]
rn = sorted(l2(a["bf16"][k], f[k]) for k in ks)
ro = sorted(l2(b["bf16"][k], f[k]) for k in ks)
print("logits new %.3e old %.3e | dx new %.3e old %.3e | median grad L2 new %.3f old %.3f | max new %.2f old %.2f" % (
    l2(a["bf16"]["logits"], f["logits"]), l2(b["bf16"]["logits"], f["logits"]), l2(a["bf16"]["dx"], f["dx"]),
    l2(b["bf16"]["dx"], f["dx"]), rn[len(rn) // 2], ro[len(ro) // 2], rn[-1], ro[-1]))

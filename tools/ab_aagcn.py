"""A/B of the AAGCN bf16 numerics between two library builds (STGCN_LIB): run config 5's model fwd+bwd at
N=16 T=300 (the test_gpu_aagcn fixture's weights/inputs) in bf16 and fp32 with the current library and save
{logits, dx, every parameter grad}.  Usage: python tools/ab_aagcn.py out.pt"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import __graft_entry__ as ge  # noqa: E402
from test_gpu_aagcn import AAGCN_ARCH, _aagcn_run  # noqa: E402

P = ge.load_package()
torch.manual_seed(1538574472)
arch = dict(AAGCN_ARCH, graph=P.PKU_MMD)
m = P.MODELS["aa-gcn"](rank=None, **arch)
with torch.no_grad():
    for name, p in m.named_parameters():
        if name.endswith(".B"):
            p.copy_(0.05 * torch.randn(p.shape))
sd0 = {k: v.clone() for k, v in m.state_dict().items()}
gen = torch.Generator().manual_seed(int(os.environ.get("AB_SEED", "0")))
x = torch.randn(16, 3, 300, 25, generator=gen)
dy = torch.randn(16, 52, 1, generator=gen)
res = {"bf16": _aagcn_run(P, arch, sd0, x, dy, "bf16"), "fp32": _aagcn_run(P, arch, sd0, x, dy, "fp32")}
torch.save(res, sys.argv[1])

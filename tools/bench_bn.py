"""Micro-benchmark of the BatchNorm row passes on the config-2 shapes (HIP-event timing), bf16:
bn_apply (BN2 + identity residual + ReLU, forward) and the fused backward passes of BN1 (mask from g, two
inputs) and BN2 (mask from y, identity residual, bias sums).   python tools/bench_bn.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

P = ge.load_package()
K = P.native
dev = "cuda:0"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for C, T in ((64, 300), (128, 150), (256, 75)):
    M = 64 * T * 25
    mk = lambda: torch.randn(64, C, T, 25, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    u, r, dy, g = mk(), mk(), mk(), mk()
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    mr = torch.stack([torch.randn(C, device=dev), torch.rand(C, device=dev) + 0.5], 1).contiguous()
    gam = torch.rand(C, device=dev) + 0.5
    out1, out2 = torch.empty_like(u), torch.empty_like(u)
    mb = M * C * 2 / 1e6
    ms = timeit(lambda: K.bn_apply(u, sc, sh, M, C, res_mode=1, r=r, relu=True, out=out1))
    print(f"bn_apply          C={C:3d}  {ms * 1e3:7.1f} us  {3 * mb / ms / 1e3:5.2f} TB/s")
    ms = timeit(lambda: K.bn_bwd_fused(dy, M, C, mask=2, mref=g, msc=sc, msh=sh, x1=g, mr1=mr, g1=gam, out1=out1))
    print(f"bn1 bwd (2 pass)  C={C:3d}  {ms * 1e3:7.1f} us  {5 * mb / ms / 1e3:5.2f} TB/s")
    ms = timeit(lambda: K.bn_bwd_fused(dy, M, C, mask=1, mref=u, x1=r, mr1=mr, g1=gam, out1=out1, out2=out2,
                                       bias_sums=True))
    print(f"bn2 bwd (2 pass)  C={C:3d}  {ms * 1e3:7.1f} us  {8 * mb / ms / 1e3:5.2f} TB/s")

"""Numerics of the joint-mix ops (amix fwd / trans (+accumulate) / attention bwd) with the current library,
saved for an A/B against another build (STGCN_LIB).  Usage: python tools/ab_amix.py out.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

P_ = ge.load_package()
K = P_.native
dev = "cuda:0"
torch.manual_seed(0)
N, T, V, P = 4, 50, 25, 3
res = {}
for C in (64, 128):
    for dt in (torch.bfloat16, torch.float32):
        A = torch.softmax(torch.randn(N, P, V, V, device=dev), -1) + 0.05 * torch.randn(N, P, V, V, device=dev)
        x = torch.randn(N, C, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
        res[f"fwd{C}{dt}"] = K.amix_fwd(x, A).float().cpu()
        dw = torch.randn(N, P * C, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
        dx = K.cl_empty(N, C, T, V, dt, dev)
        K.amix_trans(dw, A, C, dx, accumulate=False)
        res[f"trans{C}{dt}"] = dx.float().cpu()
        dx2 = x.clone()
        K.amix_trans(dw, A, C, dx2, accumulate=True)
        res[f"transacc{C}{dt}"] = dx2.float().cpu()
        ref_x = x.float()
        res[f"ref_fwd{C}{dt}"] = torch.einsum("nctv,npvw->npctw", ref_x, A).reshape(N, P * C, T, V).cpu()
        ref_dx = torch.einsum("npctw,npvw->nctv", dw.float().reshape(N, P, C, T, V), A).cpu()
        res[f"ref_trans{C}{dt}"] = ref_dx
        res[f"ref_transacc{C}{dt}"] = ref_dx + ref_x.cpu()
torch.save(res, sys.argv[1])
if len(sys.argv) > 2:
    old = torch.load(sys.argv[2])
    for k in sorted(res):
        if k.startswith("ref_"):
            continue
        ref = res["ref_" + k]
        e_new = ((res[k] - ref).norm() / ref.norm()).item()
        e_old = ((old[k] - ref).norm() / ref.norm()).item()
        print(f"{k:28s} new L2 {e_new:.3e}  old L2 {e_old:.3e}  max|new-old| {(res[k] - old[k]).abs().max().item():.3e}")

"""Micro-benchmark of config 5's (AAGCN, per-sample adjacency) graph-conv kernels at its shapes, bf16, N = 64,
V = 25, P = 3 (HIP-event timing): the A-first graph conv's joint mix (amix fwd / trans, jmix.hip), its channel
GEMM (conv_rows over P*Cin), the data-gradient GEMM, the weight gradient (wgrad1x1) and the attention
projections' weight gradient; one JSON line per shape.  Usage: python tools/bench_c5.py [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

P = ge.load_package()
K = P.native
dev = "cuda:0"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dt = torch.bfloat16


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(1e3 * s.elapsed_time(e) / reps, 1)


def cl(*shape):
    return torch.randn(*shape, device=dev).to(dt).contiguous(memory_format=torch.channels_last)


N, V, Pp = 64, 25, 3
for C, T in [(64, 300), (128, 150), (256, 75)]:
    out = {"shape": f"C={C} T={T}"}
    A = torch.rand(N, Pp, V, V, device=dev) / V
    x, dg = cl(N, C, T, V), cl(N, C, T, V)
    XA = K.amix_fwd(x, A)
    out["amix_fwd_us"] = timeit(lambda: K.amix_fwd(x, A))
    W = torch.randn(1, C, Pp * C, device=dev) / (Pp * C) ** 0.5
    wp, cp, kp = K.pack_weight(W, dt)
    out["gemm_fwd_us"] = timeit(lambda: K.conv_rows(XA, wp, Pp * C, C, cp, kp, T, T))
    b2 = torch.randn(N, V, C, device=dev)  # the graph-conv bias pushed through the per-sample A
    out["gemm_fwd_rowbias_us"] = timeit(lambda: K.conv_rows(XA, wp, Pp * C, C, cp, kp, T, T, bias=b2, bias_mode=3))
    wT, cq, kq = K.pack_weight(W.transpose(1, 2).contiguous(), dt)
    out["gemm_dgrad_us"] = timeit(lambda: K.conv_rows(dg, wT, C, Pp * C, cq, kq, T, T, trans=True))
    dXA = K.conv_rows(dg, wT, C, Pp * C, cq, kq, T, T, trans=True)
    dx = torch.empty_like(x)
    out["amix_trans_us"] = timeit(lambda: K.amix_trans(dXA, A, C, dx, False))
    out["amix_trans_acc_us"] = timeit(lambda: K.amix_trans(dXA, A, C, dx, True))
    out["amix_dA_us"] = timeit(lambda: K.amix_dA(x, dXA, A))
    out["wgrad_gcn_us"] = timeit(lambda: K.conv_wgrad(XA, dg, Pp * C, C, T, T))
    D16 = cl(N, C * 3 // 2, T, V)
    out["wgrad_attn_us"] = timeit(lambda: K.conv_wgrad(x, D16, C, C * 3 // 2, T, T))
    # attention branch (fp32 theta/phi, Nout = 2 * P * C/4 channels of one row buffer)
    No = 2 * Pp * (C // 4)
    Wp, bp = torch.randn(No, C, device=dev) / C ** 0.5, torch.randn(No, device=dev)
    out["attn_proj_us"] = timeit(lambda: K.attn_proj(x, Wp, bp))
    tp = K.attn_proj(x, Wp, bp)
    th, ph = tp[:, :No // 2], tp[:, No // 2:]
    out["attn_scores_us"] = timeit(lambda: K.attn_scores(th, ph, Pp))
    Cs = K.attn_scores(th, ph, Pp)
    dC = torch.randn_like(Cs)
    out["attn_bwd_us"] = timeit(lambda: K.attn_bwd(th, ph, Pp, Cs, dC))
    Dt = torch.randn(N, No, T, V, device=dev).contiguous(memory_format=torch.channels_last)
    out["cast_colsum_us"] = timeit(lambda: K.cast_colsum(Dt, N * T * V, No))
    print(json.dumps(out), flush=True)

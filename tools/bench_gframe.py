"""Micro-benchmark of the graph-conv kernels at the config-2 shapes (HIP-event timing, bf16, N = 64, V = 25):
forward / data grad on the joint-gathered gconv.hip vs the frame-streaming gcn_frame.hip, weight / adjacency / bias
gradients on gconv_wgrad + finish vs gconv_wgrad_frame.hip.  Prints one JSON line per shape.
Usage: python tools/bench_gframe.py [reps] [shape, e.g. 64->64]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

PKG = ge.load_package()
K = PKG.native
PKG.routing.ROUTING.gcn_frame = PKG.routing.ROUTING.gconv_wgrad_frame = True  # the opt-in kernels are timed too
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


A0 = torch.tensor(PKG.Graph(**PKG.PKU_MMD).A, dtype=torch.float32)
A = (A0 * (torch.rand(A0.shape) + 0.5)).to(dev).contiguous()
P, V = A.shape[0], A.shape[-1]
sup = K.GraphSupport(A)
N = 64
only = sys.argv[2] if len(sys.argv) > 2 else None
for Cin, Cout, T in [(64, 64, 300), (64, 128, 300), (128, 128, 150), (128, 256, 150), (256, 256, 75)]:
    if only and only != f"{Cin}->{Cout}":
        continue
    x = torch.randn(N, Cin, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    dg = torch.randn(N, Cout, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    dx = torch.empty_like(x)
    W = torch.randn(P * Cout, Cin, device=dev) / Cin ** 0.5
    b = torch.randn(P * Cout, device=dev)
    out = {"shape": f"{Cin}->{Cout} T={T}"}
    wpk, b2 = K.gconv_weights(A, W, sup, Cout, Cin, False, dt, bias=b)
    st = torch.zeros((K.gconv_row_blocks(N * T, V), wpk.shape[2], 4), device=dev)
    out["gconv_fwd_us"] = timeit(lambda: K.gconv(x, wpk, sup, Cin, Cout, bias=b2, stats=st))
    wT = K.gconv_weights(A, W, sup, Cout, Cin, True, dt)
    out["gconv_dgrad_acc_us"] = timeit(lambda: K.gconv(dg, wT, sup, Cout, Cin, trans=True, out=dx, accumulate=True))
    if K.gcn_frame_ok(sup, P, Cin, Cout, V, dt):
        img = K.pack_gcn_frame(W, P, Cout, Cin, False, dt)
        stf = torch.zeros((K.gcn_frame_row_blocks(N * T, Cout), img[1], 4), device=dev)
        out["frame_fwd_us"] = timeit(lambda: K.gcn_frame(x, A, img, Cin, Cout, bias=b2, stats=stf))
    if K.gcn_frame_ok(sup, P, Cout, Cin, V, dt):
        imgT = K.pack_gcn_frame(W, P, Cout, Cin, True, dt)
        out["frame_dgrad_acc_us"] = timeit(lambda: K.gcn_frame(dg, A, imgT, Cout, Cin, trans_a=True, out=dx,
                                                               accumulate=True))
    S = torch.empty((V, Cout), device=dev)

    def old_wgrad():
        dweff = K.gconv_wgrad(x, dg, sup, Cin, Cout, rowsum=S)
        K.gconv_finish_bias(dweff, A, W, sup, Cout, Cin, b, S)
    out["wgrad_dweff_finish_us"] = timeit(old_wgrad)
    out["wgrad_frame_us"] = timeit(lambda: K.gconv_wgrad_frame(x, dg, A, W, b))
    print(json.dumps(out), flush=True)

# the 64-channel Kt = 9 temporal conv: conv_rows (conv_wide fwd / conv_persist dgrad) vs tconv_frame.hip
if not only or only == "tcn":
    T = 300
    g = torch.randn(N, 64, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    wt = torch.randn(64, 64, 9, device=dev) * 0.05
    wtp, cp, kp = K.pack_weight(wt.permute(2, 0, 1), dt, stride=1)
    wtT, cq, kq = K.pack_weight(wt.permute(2, 1, 0), dt, stride=1, trans=True)
    sc, sh, bt = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev), torch.randn(64, device=dev)
    st0 = torch.zeros((K.row_blocks(N * T * V, 64), cp, 4), device=dev)
    st1 = torch.zeros((K.tconv_frame_row_blocks(N, T), cp, 4), device=dev)
    out = {"shape": "tcn 64->64 T=300"}
    out["conv_rows_fwd_us"] = timeit(lambda: K.conv_rows(g, wtp, 64, 64, cp, kp, T, T, Kt=9, pad=4, bias=bt, stats=st0,
                                                          pro=1, pro_a=sc, pro_b=sh))
    out["tconv_frame_fwd_us"] = timeit(lambda: K.tconv_frame(g, wtp, cp, kp, bias=bt, pro_a=sc, pro_b=sh, stats=st1))
    out["conv_rows_dgrad_us"] = timeit(lambda: K.conv_rows(g, wtT, 64, 64, cq, kq, T, T, Kt=9, pad=4, trans=True))
    out["tconv_frame_dgrad_us"] = timeit(lambda: K.tconv_frame(g, wtT, cq, kq, trans=True))
    print(json.dumps(out), flush=True)

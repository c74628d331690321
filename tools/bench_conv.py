"""Micro-benchmark of the row-conv kernels on the config-2 shapes (HIP-event timing).
Usage: python tools/bench_conv.py [reps]"""
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
    return s.elapsed_time(e) / reps


cases = [  # name, N, T, V, Cin, Cout, Kt, stride, trans, pro
    ("tcn_fwd_c64", 64, 300, 25, 64, 64, 9, 1, False, 1),
    ("tcn_dgrad_c64", 64, 300, 25, 64, 64, 9, 1, True, 0),
    ("gcn_gemm_c64", 64, 300, 25, 192, 64, 1, 1, False, 0),
    ("tcn_fwd_c128", 64, 150, 25, 128, 128, 9, 1, False, 1),
    ("tcn_fwd_c256", 64, 75, 25, 256, 256, 9, 1, False, 1),
    ("gcn_gemm_c256", 64, 75, 25, 768, 256, 1, 1, False, 0),
    ("tcn_dgrad_c128", 64, 150, 25, 128, 128, 9, 1, True, 0),
    ("tcn_dgrad_c256", 64, 75, 25, 256, 256, 9, 1, True, 0),
    ("tcn_fwd_s2_c128", 64, 300, 25, 128, 128, 9, 2, False, 1),
    ("gcn_gemm_c128", 64, 150, 25, 384, 128, 1, 1, False, 0),
    ("tcn_dgrad_s2_c128", 64, 300, 25, 128, 128, 9, 2, True, 0),
    ("res_dgrad_s2_c128", 64, 300, 25, 128, 64, 1, 2, True, 0),
]
only = sys.argv[2] if len(sys.argv) > 2 else None
for name, N, T, V, Cin, Cout, Kt, s, trans, pro in cases:
    if only and name != only:
        continue
    pad = (Kt - 1) // 2
    T_out = T if s == 1 else (T - 1) // s + 1
    Ti, To = (T_out, T) if trans else (T, T_out)
    x = torch.randn(N, Cin, Ti, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    w = torch.randn(Kt, Cout, Cin, device=dev) * 0.05
    wp, cp, kp = K.pack_weight(w, dt, stride=s, trans=trans)
    sc = torch.rand(Cin, device=dev) + 0.5
    sh = torch.randn(Cin, device=dev)
    b = torch.randn(Cout, device=dev)
    kw = dict(pro=1, pro_a=sc, pro_b=sh) if pro else {}
    if not trans:  # forward convs feed a BatchNorm: epilogue partial statistics
        kw["stats"] = torch.zeros((K.row_blocks(N * To * V, Cout), cp, 4), device=dev)
    f = lambda: K.conv_rows(x, wp, Cin, Cout, cp, kp, Ti, To, Kt=Kt, stride=s, pad=pad, trans=trans, bias=None if trans else b, **kw)
    ms = timeit(f)
    flops = 2.0 * N * To * V * Cin * Cout * Kt
    byts = (N * Ti * V * Cin + N * To * V * Cout) * 2
    print(f"{name:16s} {ms*1e3:9.1f} us  {flops/ms/1e9:8.1f} TFLOP/s  {byts/ms/1e6:8.1f} GB/s", flush=True)

# the 64-channel temporal conv kernels outside conv_rows: tconv_frame (forward with the BN1 prologue, bias and
# BN partials; data grad) and layer_fused's g-input mode
for name in ("tf_fwd_c64", "tf_dgrad_c64"):
    if only and name != only:
        continue
    N, T, V, C = 64, 300, 25, 64
    x = torch.randn(N, C, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    w = torch.randn(9, C, C, device=dev) * 0.05
    trans = name == "tf_dgrad_c64"
    wp, cp, kp = K.pack_weight(w, dt, stride=1, trans=trans)
    sc = torch.rand(C, device=dev) + 0.5
    sh = torch.randn(C, device=dev)
    b = torch.randn(C, device=dev)
    if name == "tf_fwd_c64":
        st = torch.zeros((K.tconv_frame_row_blocks(N, T), cp, 4), device=dev)
        f = lambda: K.tconv_frame(x, wp, cp, kp, bias=b, pro_a=sc, pro_b=sh, stats=st)
    else:
        f = lambda: K.tconv_frame(x, wp, cp, kp, trans=True)
    ms = timeit(f)
    flops = 2.0 * N * T * V * C * C * 9
    print(f"{name:16s} {ms*1e3:9.1f} us  {flops/ms/1e9:8.1f} TFLOP/s  {4*N*T*V*C/ms/1e6:8.1f} GB/s", flush=True)

wcases = [  # name, N, T, V, Cin, Cout, Kt, stride, pro
    ("tcn_wgrad_c64", 64, 300, 25, 64, 64, 9, 1, 1),
    ("tcn_wgrad_c128", 64, 150, 25, 128, 128, 9, 1, 1),
    ("tcn_wgrad_c256", 64, 75, 25, 256, 256, 9, 1, 1),
    ("tcn_wgrad_s2_c128", 64, 300, 25, 128, 128, 9, 2, 1),
    ("gcn_wgrad_c64", 64, 300, 25, 192, 64, 1, 1, 0),
    ("gcn_wgrad_c256", 64, 75, 25, 768, 256, 1, 1, 0),
    ("res_wgrad_s2_c128", 64, 300, 25, 64, 128, 1, 2, 0),
]
for name, N, T, V, Cin, Cout, Kt, s, pro in wcases:
    if only and name != only:
        continue
    pad = (Kt - 1) // 2
    T_out = (T + 2 * pad - Kt) // s + 1
    x = torch.randn(N, Cin, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, Cout, T_out, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    sc = torch.rand(Cin, device=dev) + 0.5
    sh = torch.randn(Cin, device=dev)
    kw = dict(pro=1, pro_a=sc, pro_b=sh) if pro else {}
    dw = torch.zeros((Kt, Cout, Cin), device=dev)
    f = lambda: K.conv_wgrad(x, dy, Cin, Cout, T, T_out, Kt=Kt, stride=s, pad=pad, dw=dw, **kw)
    ms = timeit(f)
    flops = 2.0 * N * T_out * V * Cin * Cout * Kt
    byts = (N * T * V * Cin + N * T_out * V * Cout) * 2
    print(f"{name:18s} {ms*1e3:9.1f} us  {flops/ms/1e9:8.1f} TFLOP/s  {byts/ms/1e6:8.1f} GB/s", flush=True)

# joint-gathered graph conv (gconv.hip) on the PKU-MMD graph: fwd (S lists) and data grad (R lists),
# algorithmic flops = 2 * N*T * nnz(support) * Cin * Cout
A0 = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32, device=dev)
sup = K.GraphSupport(A0)
gcases = [("gconv_fwd_c64", 64, 300, 64, 64), ("gconv_fwd_c128", 64, 150, 128, 128),
          ("gconv_fwd_c256", 64, 75, 256, 256), ("gconv_fwd_64to128", 64, 300, 64, 128),
          ("gconv_fwd_128to256", 64, 150, 128, 256)]
for name, N, T, Cin, Cout in gcases:
    if only and not name.startswith(only):
        continue
    Pp, V = A0.shape[0], A0.shape[-1]
    W = torch.randn(Pp * Cout, Cin, device=dev) / Cin ** 0.5
    x = torch.randn(N, Cin, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    dg = torch.randn(N, Cout, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    wpk = K.gconv_weights(A0, W, sup, Cout, Cin, False, dt)
    wT = K.gconv_weights(A0, W, sup, Cout, Cin, True, dt)
    b2 = K.gcn_bias(A0, torch.randn(Pp * Cout, device=dev), N, Cout)
    st = torch.zeros((K.gconv_row_blocks(N * T, V), wpk.shape[2], 4), device=dev)
    flops = 2.0 * N * T * sup.nnz * Cin * Cout
    byts = (N * T * V * (Cin + Cout)) * 2
    for tag, f in (("", lambda: K.gconv(x, wpk, sup, Cin, Cout, bias=b2, stats=st)),
                   ("_dgrad", lambda: K.gconv(dg, wT, sup, Cout, Cin, trans=True))):
        ms = timeit(f)
        print(f"{name + tag:22s} {ms*1e3:9.1f} us  {flops/ms/1e9:8.1f} TFLOP/s  {byts/ms/1e6:8.1f} GB/s", flush=True)
    ms = timeit(lambda: K.gconv_wgrad(x, dg, sup, Cin, Cout))
    print(f"{name.replace('fwd', 'wgrad'):22s} {ms*1e3:9.1f} us  {flops/ms/1e9:8.1f} TFLOP/s", flush=True)


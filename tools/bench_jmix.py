"""Micro-benchmark of the dense joint-mix kernels (jmix.hip) at config-5 shapes: amix fwd / trans (per-sample
A, bf16, N=64 T=300 C=64 and T=75 C=256) and the attention-backward mix (fp32, 48 channels).  HIP-event
timing; algorithmic bytes = input rows read once + output rows written once.
usage: python tools/bench_jmix.py [reps] [case]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

P_ = ge.load_package()
K = P_.native
dev = "cuda:0"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
only = sys.argv[2] if len(sys.argv) > 2 else None


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


N, V, P = 64, 25, 3
for name, T, C in (("c64", 300, 64), ("c256", 75, 256)):
    A = torch.softmax(torch.randn(N, P, V, V, device=dev), -1)
    x = torch.randn(N, C, T, V, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dw = torch.randn(N, P * C, T, V, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dx = K.cl_empty(N, C, T, V, torch.bfloat16, dev)
    M = N * T * V
    for case, fn, byts in ((f"amix_fwd_{name}", lambda: K.amix_fwd(x, A), M * 4 * C * 2),
                           (f"amix_trans_{name}", lambda: K.amix_trans(dw, A, C, dx, accumulate=False), M * 4 * C * 2),
                           (f"amix_trans_acc_{name}", lambda: K.amix_trans(dw, A, C, dx, accumulate=True),
                            M * 5 * C * 2)):
        if only and case != only:
            continue
        ms = timeit(fn)
        print(f"{case:22s} {ms * 1e3:8.1f} us  {byts / ms / 1e6:8.1f} GB/s", flush=True)
T, ce = 300, 16
th = torch.randn(N, P * ce, T, V, device=dev).contiguous(memory_format=torch.channels_last)
ph = torch.randn(N, P * ce, T, V, device=dev).contiguous(memory_format=torch.channels_last)
C = K.attn_scores(th, ph, P)
dC = torch.randn_like(C)
if not only or only == "attn_bwd":
    ms = timeit(lambda: K.attn_bwd(th, ph, P, C, dC))
    byts = 4 * N * T * V * P * ce * 4
    print(f"{'attn_bwd':22s} {ms * 1e3:8.1f} us  {byts / ms / 1e6:8.1f} GB/s", flush=True)

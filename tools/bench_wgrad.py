"""Micro-benchmark of the temporal-conv weight gradient (stgcn_conv_wgrad: wgrad_ring / wgrad_wide / wgrad_tile by
shape) at the config-2 shapes, N = 64, bf16, HIP-event timing of the whole C-ABI call (kernel + slab reduction).
Usage: python tools/bench_wgrad.py [reps] [shape filter, e.g. 64s1]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

K = ge.load_package().native
dev = "cuda:0"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
only = sys.argv[2] if len(sys.argv) > 2 else None
N, V = 64, 25


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


for C, stride, T in [(64, 1, 300), (128, 1, 150), (256, 1, 75), (128, 2, 300), (256, 2, 150)]:
    tag = f"{C}s{stride}"
    if only and only != tag:
        continue
    To = (T - 1) // stride + 1
    x = torch.randn(N, C, T, V, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, C, To, V, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    out = {"shape": tag}
    for pro in (1, 0):
        kw = dict(Kt=9, stride=stride, pad=4, pro=pro, pro_a=sc if pro else None, pro_b=sh if pro else None)
        us = timeit(lambda: K.conv_wgrad_w(x, dy, C, C, T, To, **kw))
        out[f"pro{pro}_us"] = us
        out[f"pro{pro}_tflops"] = round(2.0 * N * To * V * C * C * 9 / us / 1e6, 1)
    print(json.dumps(out), flush=True)

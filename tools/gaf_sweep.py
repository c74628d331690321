"""gcn_af.hip time vs frames (setup intercept and per-tile slope): python tools/gaf_sweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

P = ge.load_package()
K = P.native
dev = "cuda:0"
A0 = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32, device=dev)
sup = K.GraphSupport(A0)
Pp, V = A0.shape[0], A0.shape[-1]
W = torch.randn(Pp * 64, 64, device=dev) / 8
b2 = K.gcn_bias(A0, torch.randn(Pp * 64, device=dev), 1, 64)


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for NT in (4, 512, 2048, 4096, 8192, 19200):
    x = torch.randn(1, 64, NT, V, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    st = torch.zeros((K.gcn_af_blocks(NT, V), 64, 4), device=dev)
    t_f = timeit(lambda: K.gcn_af(x, A0, W, sup, bias=b2, stats=st))
    t_n = timeit(lambda: K.gcn_af(x, A0, W, sup))
    t_d = timeit(lambda: K.gcn_af(x, A0, W, sup, trans=True))
    print(f"NT {NT:6d} blocks {K.gcn_af_blocks(NT, V):4d}  fwd+bias+stats {t_f:7.1f} us  fwd {t_n:7.1f} us  "
          f"dgrad {t_d:7.1f} us", flush=True)

"""Host cost (µs per call, no GPU sync inside the loop) of the pieces every kernel wrapper pays."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
K = pkg.native
L = sys.modules[pkg.__name__ + "._lib"]
dev = torch.device("cuda", 0)
part = torch.zeros((1920, 64, 4), device=dev)
g = torch.ones(64, device=dev)
b = torch.zeros(64, device=dev)


def t(name, fn, n=2000):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    print(f"{name:40s} {dt:7.2f} us", flush=True)


t("torch.cuda.current_stream().cuda_stream", lambda: torch.cuda.current_stream().cuda_stream)
t("torch._C._cuda_getCurrentRawStream(0)", lambda: torch._C._cuda_getCurrentRawStream(0))
t("L.stream()", L.stream)
t("torch.empty(64)", lambda: torch.empty(64, device=dev))
t("torch.empty((1920,64,4))", lambda: torch.empty((1920, 64, 4), device=dev))
t("torch.zeros(64)", lambda: torch.zeros(64, device=dev))
t("tensor.data_ptr()", lambda: part.data_ptr())
t("p.detach().float()", lambda: g.detach().float())
t("K.bn_finalize", lambda: K.bn_finalize(part, 1920, 64, 64, g, b))
t("raw stgcn_bn_finalize (ctypes)", lambda: L.lib().stgcn_bn_finalize(part.data_ptr(), 1920, 64, 64, g.data_ptr(), b.data_ptr(), 1e-5, part.data_ptr(), b.data_ptr(), b.data_ptr(), L.stream()))
t("torch add_ (1 launch)", lambda: b.add_(1.0))

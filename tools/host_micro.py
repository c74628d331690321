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

# kernel wrappers at a small shape (host cost dominates)
x = torch.randn(2, 64, 16, 25, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w3 = torch.randn(9, 64, 64, device=dev)
wp, cp, kp = K.pack_weight(w3, torch.bfloat16)
A0 = torch.tensor(pkg.Graph(**pkg.PKU_MMD).A, dtype=torch.float32, device=dev)
sup = K.GraphSupport(A0)
Wg = torch.randn(3 * 64, 64, device=dev)
wpk = K.gconv_weights(A0, Wg, sup, 64, 64, False, torch.bfloat16)
bg = torch.randn(3 * 64, device=dev)
b2 = K.gcn_bias(A0, bg, 2, 64)
sc = torch.ones(64, device=dev)
u = K.conv_rows(x, wp, 64, 64, cp, kp, 16, 16, Kt=9, pad=4)
t("K.pack_weight (Kt=9, frag)", lambda: K.pack_weight(w3, torch.bfloat16), 500)
t("K.gconv_weights", lambda: K.gconv_weights(A0, Wg, sup, 64, 64, False, torch.bfloat16), 500)
t("K.gcn_bias", lambda: K.gcn_bias(A0, bg, 2, 64), 500)
t("K.gconv", lambda: K.gconv(x, wpk, sup, 64, 64, bias=b2), 500)
t("K.conv_rows (Kt=9)", lambda: K.conv_rows(x, wp, 64, 64, cp, kp, 16, 16, Kt=9, pad=4, pro=1, pro_a=sc, pro_b=sc), 500)
t("K.bn_apply", lambda: K.bn_apply(u, sc, sc, 2 * 16 * 25, 64, res_mode=1, r=x), 500)
t("K.zeros_arena (3 shapes)", lambda: K.zeros_arena(dev, (100, 64, 4), (100, 64, 4), (100, 64, 4)), 500)
layer = pkg.StgcnLayer(64, 64, (9, 25), 3, 25, stride=1).to(dev)
pkg.set_compute_dtype(layer, "bf16")
xg = x.detach().clone().requires_grad_(True)
t("StgcnLayer fwd (training path)", lambda: layer(xg, A0), 200)
y = layer(xg, A0)
gy = torch.randn_like(y)
t("StgcnLayer fwd+bwd (training path)", lambda: torch.autograd.backward(layer(xg, A0), gy), 200)

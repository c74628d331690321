"""Micro-benchmark of the LayerNorm([C,1,V]) kernels (ln.hip) at the config-2 activation shapes, bf16, N = 64:
ln_stats, ln_apply (h = relu(LN(g)); y = relu(LN(u) + x); y = relu(LN(u) + LN_r(r))), ln_bwd (mask from the
output, with dgamma/dbeta; mask 2 = relu(LN(x))).  HIP-event timing; prints one JSON line per shape with the
achieved GB/s of each (algorithmic bytes: every activation read / written once)."""
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


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return 1e3 * s.elapsed_time(e) / reps


N, V = 64, 25
for C, T in [(64, 300), (128, 150), (256, 75)]:
    F = N * T
    M = F * V
    act = M * C * 2
    mk = lambda: torch.randn(N, C, T, V, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g, u, r, x, dy = mk(), mk(), mk(), mk(), mk()
    gam, bet = torch.rand(C * V, device=dev) + 0.5, torch.randn(C * V, device=dev)
    out = {"shape": f"C={C} T={T}", "activation_MB": round(act / 1e6, 1)}
    st = K.ln_stats(g, F, V, C)
    rst = K.ln_stats(r, F, V, C)
    res = {}
    res["stats"] = (timeit(lambda: K.ln_stats(g, F, V, C)), 1)
    h = torch.empty_like(g)
    res["apply_h"] = (timeit(lambda: K.ln_apply(g, st, gam, bet, M, V, C, relu=True, out=h)), 2)
    res["apply_res1"] = (timeit(lambda: K.ln_apply(u, st, gam, bet, M, V, C, res_mode=1, r=x, out=h)), 3)
    res["apply_res2"] = (timeit(lambda: K.ln_apply(u, st, gam, bet, M, V, C, res_mode=2, r=r, rst=rst, rg=gam, rb=bet,
                                                  out=h)), 3)
    dx = torch.empty_like(g)
    dgb = torch.zeros((2, C * V), device=dev)
    res["bwd_mask1_dgb"] = (timeit(lambda: K.ln_bwd(dy, u, st, gam, bet, F, V, C, dx, mask=1, mref=x, dgb=dgb)), 4)
    res["bwd_mask2_dgb"] = (timeit(lambda: K.ln_bwd(dy, g, st, gam, bet, F, V, C, dx, mask=2, dgb=dgb)), 3)
    res["bwd_nodgb"] = (timeit(lambda: K.ln_bwd(dy, g, st, gam, bet, F, V, C, dx)), 3)
    for k, (us, n) in res.items():
        out[k + "_us"] = round(us, 1)
        out[k + "_GBps"] = round(n * act / (us * 1e3), 0)
    print(json.dumps(out), flush=True)

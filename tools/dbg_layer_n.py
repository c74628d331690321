"""bf16 StgcnLayer gradients vs the fp32 HIP path at growing N (T fixed): error growth and run-to-run
determinism of each gradient.  usage: dbg_layer_n.py cin cout stride T N1,N2,..."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
P = ge.load_package()
DEV = "cuda:0"
cin, cout, stride, T = (int(v) for v in sys.argv[1:5])
A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32)
for N in [int(v) for v in sys.argv[5].split(",")]:
    torch.manual_seed(300 + cin + cout)
    layer = P.StgcnLayer(cin, cout, (9, 25), 3, 25, stride=stride, normalization="BatchNorm")
    M = 1 + 0.1 * torch.randn(3, 25, 25)
    x = torch.randn(N, cin, T, 25)
    dy = torch.randn(N, cout, (T - 1) // stride + 1, 25)
    layer = layer.to(DEV)
    res = {}
    for tag, dt in (("f32", "fp32"), ("b1", "bf16"), ("b2", "bf16")):
        P.set_compute_dtype(layer, dt)
        layer.zero_grad(set_to_none=True)
        xg = x.to(DEV).requires_grad_(True)
        Ag = (A * M).to(DEV).requires_grad_(True)
        y = layer(xg, Ag)
        y.backward(dy.to(DEV))
        g = {"y": y.detach().float(), "dx": xg.grad.float(), "dA": Ag.grad.float()}
        g.update({k: p.grad.detach().float().clone() for k, p in layer.named_parameters()})
        res[tag] = g
    line = [f"N={N}"]
    for k in res["f32"]:
        r = res["f32"][k]
        e = (res["b1"][k] - r).norm() / r.norm().clamp_min(1e-30)
        em = (res["b1"][k] - r).abs().max() / r.abs().max().clamp_min(1e-30)
        det = torch.equal(res["b1"][k], res["b2"][k])
        line.append(f"{k}: L2 {e:.1e} max {em:.1e}{'' if det else ' NONDET'}")
    print("\n  ".join(line), flush=True)

"""Parity of the HIP path with the reference, on the MI355X.

* Golden fixtures (reference outputs, tests/golden/*.npz): the HIP fp32 path must match forward
  AND backward within the north-star tolerance, max|got - ref| <= 1e-3 * max|ref|.
* Larger shapes: HIP fp32 vs the CPU oracle (oracle/stgcn_oracle.py, itself pinned to the
  fixtures) on identical seeded inputs; bf16 path vs the oracle within 3e-2 (bf16 storage of
  activations between kernels, fp32 accumulation).
"""
import numpy as np
import pytest
import torch

from conftest import assert_close, assert_grad_close, grad_floor, load_golden, sub
from oracle import stgcn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-3  # BASELINE.json north_star: 1e-3 fp32 relative


@pytest.fixture(scope="module")
def P(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg


def _load(module, sd):
    missing, unexpected = module.load_state_dict({k: v.float() for k, v in sd.items()}, strict=True), None
    return module


LAYER_CASES = ["bn_s1", "bn_s2", "ln_s1", "ln_s2", "bn_c64", "ln_k69", "bn_nores"]


@pytest.mark.parametrize("case", LAYER_CASES)
def test_stgcn_layer_golden(P, case):
    d = load_golden("stgcn_layer_" + case)
    cin, cout, stride, kt, is_ln, residual = [int(v) for v in d["cfg"]]
    layer = P.StgcnLayer(cin, cout, (kt, 25), 3, 25, stride=stride, residual=bool(residual),
                         normalization="LayerNorm" if is_ln else "BatchNorm")
    layer.load_state_dict(sub(d, "sd/"), strict=True)
    layer = layer.to(DEV)
    x = d["x"].to(DEV).requires_grad_(True)
    Aeff = (d["A"] * d["M"]).to(DEV).requires_grad_(True)
    y = layer(x, Aeff)
    assert_close(y, d["y"], TOL, "y")
    y.backward(d["dy"].to(DEV))
    assert_close(x.grad, d["dx"], TOL, "dx")
    assert_close(Aeff.grad, d["dAeff"], TOL, "dAeff")
    grads = sub(d, "grad/")
    named = dict(layer.named_parameters())
    for k, g in grads.items():
        assert_close(named[k].grad, g, TOL, k, grad_floor(grads, k))


@pytest.mark.parametrize("shared", [False, True])
def test_tgcn_golden(P, shared):
    d = load_golden("tgcn_batched")
    m = P.ConvTemporalGraphical(16, 24, 25, 3)
    m.load_state_dict(sub(d, "sd/"))
    m = m.to(DEV)
    x = d["x"].to(DEV).requires_grad_(True)
    A = (d["A_shared"] if shared else d["A"]).to(DEV).requires_grad_(True)
    y = m(x, A)
    sfx, gp = ("_shared", "grad_shared/") if shared else ("", "grad/")
    assert_close(y, d["y" + sfx], TOL, "y")
    y.backward(d["dy"].to(DEV))
    assert_close(x.grad, d["dx" + sfx], TOL, "dx")
    assert_close(A.grad, d["dA" + sfx], TOL, "dA")
    assert_close(m.conv.weight.grad, d[gp + "conv.weight"], TOL, "dw")
    assert_close(m.conv.bias.grad, d[gp + "conv.bias"], TOL, "db")


def test_norms_golden(P):
    d = load_golden("norms")
    ln = P.LayerNorm([8, 1, 25])
    ln.load_state_dict(sub(d, "ln_sd/"))
    ln = ln.to(DEV)
    x = d["ln_x"].to(DEV).requires_grad_(True)
    y = ln(x)
    assert_close(y, d["ln_y"], TOL, "ln y")
    y.backward(d["ln_dy"].to(DEV))
    assert_close(x.grad, d["ln_dx"], TOL, "ln dx")
    assert_close(ln.weight.grad, d["ln_grad/weight"], TOL, "ln dw")
    bn = P.BatchNorm1d(75)
    bn.load_state_dict(sub(d, "bn_sd/"))
    bn = bn.to(DEV)
    x = d["bn_x"].to(DEV).requires_grad_(True)
    y = bn(x)
    assert_close(y, d["bn_y"], TOL, "bn y")
    y.backward(d["bn_dy"].to(DEV))
    assert_close(x.grad, d["bn_dx"], TOL, "bn dx")
    assert_close(bn.norm.weight.grad, d["bn_grad/norm.weight"], TOL, "bn dw")


@pytest.mark.parametrize("case", ["stgcn_bn_1layer", "stgcn_bn_1layer_t64", "stgcn_ln_1layer_t64", "stgcn_bn_9layer_narrow",
                                  "stgcn_ln_9layer_narrow_k69"])
def test_stgcn_model_golden(P, case):
    d = load_golden("model_" + case)
    m = P.MODELS["st-gcn"](rank=None, **d["arch"])
    m.load_state_dict(sub(d, "sd/"), strict=True)
    m = m.to(DEV)
    x = d["x"].to(DEV).requires_grad_(True)
    y = m(x)
    assert_close(y, d["y"], TOL, "y")
    y.backward(d["dy"].to(DEV))
    assert_close(x.grad, d["dx"], TOL, "dx")
    grads = sub(d, "grad/")
    named = dict(m.named_parameters())
    for k, g in grads.items():
        assert_close(named[k].grad, g, TOL, k, grad_floor(grads, k))


@pytest.mark.parametrize("norm", ["BatchNorm", "LayerNorm"])
@pytest.mark.parametrize("cin,cout,stride", [(64, 64, 1), (64, 128, 2), (256, 256, 1)])
def test_layer_vs_oracle_larger(P, norm, cin, cout, stride):
    """N=4, T=64 (config-2 channel widths) fp32 HIP vs the CPU oracle, forward and backward."""
    torch.manual_seed(7)
    N, T = 4, 64
    A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32)
    layer = P.StgcnLayer(cin, cout, (9, 25), 3, 25, stride=stride, normalization=norm)
    with torch.no_grad():
        for name, p in layer.named_parameters():
            if "tcn.0" in name or "tcn.3" in name or "residual.1" in name:
                p.add_(0.1 * torch.randn(p.shape))
    M = 1 + 0.1 * torch.randn(3, 25, 25)
    x = torch.randn(N, cin, T, 25)
    dy = torch.randn(N, cout, (T - 1) // stride + 1, 25)
    sd = {k: v.clone().requires_grad_(True) for k, v in layer.state_dict().items()}
    xr = x.clone().requires_grad_(True)
    Ar = (A * M).requires_grad_(True)
    ref = O.stgcn_layer(xr, Ar, sd, "", 9, stride, True, norm)
    ref.backward(dy)
    layer = layer.to(DEV)
    xg = x.to(DEV).requires_grad_(True)
    Ag = (A * M).to(DEV).requires_grad_(True)
    y = layer(xg, Ag)
    y.backward(dy.to(DEV))
    assert_close(y, ref, TOL, "y")
    assert_grad_close(xg.grad, xr.grad, TOL, "dx")
    assert_grad_close(Ag.grad, Ar.grad, TOL, "dA", reduction=True)
    named = dict(layer.named_parameters())
    grads = {k: v.grad for k, v in sd.items() if v.grad is not None}
    for k, g in grads.items():
        assert_grad_close(named[k].grad, g, TOL, k, grad_floor(grads, k), reduction=True)


@pytest.mark.parametrize("cin,cout,stride", [(64, 64, 1), (64, 128, 2), (128, 64, 1)])
def test_layer_bf16_vs_oracle(P, cin, cout, stride):
    """bf16 perf path of one BatchNorm layer at config-2 widths on the 25-joint graph vs the fp32 oracle: forward
    and every gradient within bf16 tolerance (graph conv on the gathered gconv.hip)."""
    torch.manual_seed(5)
    N, T = 3, 40
    A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32)
    layer = P.StgcnLayer(cin, cout, (9, 25), 3, 25, stride=stride, normalization="BatchNorm")
    M = 1 + 0.1 * torch.randn(3, 25, 25)
    x = torch.randn(N, cin, T, 25)
    dy = torch.randn(N, cout, (T - 1) // stride + 1, 25)
    sd = {k: v.clone().requires_grad_(True) for k, v in layer.state_dict().items()}
    xr = x.clone().requires_grad_(True)
    Ar = (A * M).requires_grad_(True)
    ref = O.stgcn_layer(xr, Ar, sd, "", 9, stride, True, "BatchNorm")
    ref.backward(dy)
    layer = P.set_compute_dtype(layer.to(DEV), "bf16")
    xg = x.to(DEV).requires_grad_(True)
    Ag = (A * M).to(DEV).requires_grad_(True)
    y = layer(xg, Ag)
    y.backward(dy.to(DEV))
    tol = 4e-2
    assert_close(y.float(), ref, tol, "y")
    assert_grad_close(xg.grad, xr.grad, tol, "dx")
    assert_grad_close(Ag.grad, Ar.grad, tol, "dA", reduction=True)
    named = dict(layer.named_parameters())
    grads = {k: v.grad for k, v in sd.items() if v.grad is not None}
    for k, g in grads.items():
        if float(g.abs().max()) < 1e-3 * grad_floor(grads, k):
            # a conv bias feeding a batch-statistics BatchNorm: its true gradient is 0 (the reference's
            # is fp32 rounding noise, ours the sum of bf16-rounded BN input grads over all rows)
            assert float(named[k].grad.abs().max()) < 0.3 * grad_floor(grads, k), k
            continue
        assert_grad_close(named[k].grad, g, tol, k, grad_floor(grads, k), reduction=True)


def test_model_bf16_vs_oracle(P):
    """bf16 perf path, 9-layer as_is model (narrow widths), vs the fp32 oracle: 3e-2 relative."""
    d = load_golden("model_stgcn_bn_9layer_narrow")
    m = P.MODELS["st-gcn"](rank=None, **d["arch"])
    m.load_state_dict(sub(d, "sd/"), strict=True)
    m = m.to(DEV).set_compute_dtype("bf16")
    y = m(d["x"].to(DEV))
    assert_close(y, d["y"], 3e-2, "bf16 model y")

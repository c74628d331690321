"""The fused ST-GCN layer (layer_fused.hip, the BASELINE north_star kernel): a LayerNorm StgcnLayer as ONE kernel —
graph conv + LN1 + ReLU + temporal conv + LN2 + residual + ReLU with g and h kept on chip.

* kernel level: stgcn_layer_fused_fwd through the C-ABI against the fp32 oracle on the same bf16-rounded operands
  (oracle.tgcn = tgcn.py:58-79, layernorm_cv = layernorm.py:22-28, F.conv2d = stgcn.py:154-159) at a short trial
  (a partial last step, padding frames at both ends) and at the bench shape (N=64 T=300);
* layer / model level: StgcnLayer and the config-2 Model in inference (no autograd) and training (routing
  fused_ln_train) — the paths that route through the fused kernel — against the fp32 oracle (stgcn.py:80-97,
  181-193), bf16 tolerance; BatchNorm layers take the unfused route (no one-kernel BatchNorm form: BN1's batch
  statistics need all of g first).
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import assert_close
from oracle import stgcn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
BF = torch.bfloat16


@pytest.fixture(scope="module")
def P(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg


def cl(x, dtype=torch.float32):
    return x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)


def rb(t):
    return t.to(BF).float()


def _graph(P):
    A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32)
    g = torch.Generator().manual_seed(7)
    return A * (1 + 0.1 * torch.randn(A.shape, generator=g))  # edge importance applied


def _count_fused(P, monkeypatch):
    calls = []
    orig = P.native.layer_fused

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(P.native, "layer_fused", spy)
    monkeypatch.setattr(P.routing.ROUTING, "fused_inference", True)  # whatever the environment chose
    return calls


def test_bn_inference_unfused_route(P, monkeypatch):
    """A BatchNorm layer's inference forward takes the unfused route (there is no one-kernel BatchNorm form) and
    matches the fp32 oracle."""
    calls = _count_fused(P, monkeypatch)
    torch.manual_seed(4)
    N, T, V = 4, 64, 25
    A = _graph(P)
    layer = P.StgcnLayer(64, 64, (9, V), 3, V, stride=1, normalization="BatchNorm")
    sd = {k: v.clone() for k, v in layer.state_dict().items()}
    x = torch.randn(N, 64, T, V)
    ref = O.stgcn_layer(x, A, sd, "", 9, 1, True, "BatchNorm")
    layer = layer.to(DEV)
    P.set_compute_dtype(layer, "bf16")
    with torch.no_grad():
        y = layer(x.to(DEV), A.to(DEV))
    torch.cuda.synchronize()
    assert not calls, "BatchNorm inference took the (LayerNorm-only) fused kernel"
    assert_close(y.float().cpu(), ref, 3e-2, "unfused inference layer")


@pytest.mark.parametrize("norm", ["BatchNorm", "LayerNorm"])
@pytest.mark.parametrize("residual", [True, False])
def test_stgcn_layer_inference_fused(P, monkeypatch, residual, norm):
    """StgcnLayer (64 -> 64, stride 1) under no_grad: LayerNorm takes the one-kernel layer, BatchNorm the unfused
    route; vs the fp32 oracle."""
    calls = _count_fused(P, monkeypatch)
    torch.manual_seed(3)
    N, T, V = 8, 100, 25
    A = _graph(P)
    layer = P.StgcnLayer(64, 64, (9, V), 3, V, stride=1, residual=residual, normalization=norm)
    sd = {k: v.clone() for k, v in layer.state_dict().items()}
    g = torch.Generator().manual_seed(5)
    for k in sd:  # non-trivial affines
        if k.endswith("weight") and sd[k].dim() == 1:
            sd[k] = 1 + 0.2 * torch.randn(sd[k].shape, generator=g)
        elif k.endswith("bias"):
            sd[k] = 0.1 * torch.randn(sd[k].shape, generator=g)
    layer.load_state_dict(sd)
    x = torch.randn(N, 64, T, V)
    ref = O.stgcn_layer(x, A, sd, "", 9, 1, residual, norm)
    layer = layer.to(DEV)
    P.set_compute_dtype(layer, "bf16")
    with torch.no_grad():
        y = layer(x.to(DEV), A.to(DEV))
    torch.cuda.synchronize()
    assert len(calls) == (1 if norm == "LayerNorm" else 0), f"fused kernel calls {calls}"
    assert_close(y.float().cpu(), ref, 3e-2, "inference layer")


@pytest.mark.parametrize("T", [300, 37])
def test_layer_fused_ln_kernel(P, T):
    """The LayerNorm whole-layer kernel through the C-ABI at the bench shape (N=64: several runs per sample)
    and a short trial (partial last step): y vs the fp32 oracle on the same bf16-rounded operands."""
    K = P.native
    torch.manual_seed(T)
    N, V, C = (64 if T == 300 else 3), 25, 64
    A = _graph(P)
    Pp = A.shape[0]
    x = rb(torch.randn(N, C, T, V))
    wg = rb(torch.randn(Pp * C, C, 1, 1) / C ** 0.5)
    bg = torch.randn(Pp * C) * 0.1
    wt = rb(torch.randn(C, C, 9, 1) / (9 * C) ** 0.5)
    bt = torch.randn(C) * 0.1
    g1, b1, g2, b2 = (1 + 0.2 * torch.randn(C, 1, V), 0.2 * torch.randn(C, 1, V), 1 + 0.2 * torch.randn(C, 1, V),
                      0.2 * torch.randn(C, 1, V))
    h = torch.relu(O.layernorm_cv(O.tgcn(x, wg, bg, A), g1, b1))
    ref = torch.relu(O.layernorm_cv(F.conv2d(rb(h), wt, bt, padding=(4, 0)), g2, b2) + x)
    A_d = A.to(DEV)
    bias2d = K.gcn_bias(A_d, bg.to(DEV), N, C)
    wgf = wg.view(Pp, C, C).permute(1, 0, 2).reshape(C, Pp * C).to(DEV)
    wimg, _, _ = K.pack_gcn_weight(wgf, BF)
    wtp, _, _ = K.pack_weight(wt.squeeze(-1).permute(2, 0, 1).to(DEV), BF, stride=1)
    vc = lambda t: t.reshape(C, V).t().contiguous().to(DEV)  # noqa: E731
    y = K.layer_fused(cl(x, BF), A_d, wimg, bias2d, wtp, bt.to(DEV), (vc(g1), vc(b1), vc(g2), vc(b2)), residual=True)
    assert_close(y.float(), ref, 3e-2, "fused LN layer")


@pytest.mark.parametrize("norm", ["BatchNorm", "LayerNorm"])
def test_model_inference_fused_config2(P, monkeypatch, norm):
    """The config-2 model (9 layers, N=16 T=300; as_is BatchNorm and the ln/ LayerNorm variant) in
    inference: the LayerNorm model's layers 0-2 run as the one-kernel layer (the BatchNorm model's unfused);
    logits vs the oracle."""
    calls = _count_fused(P, monkeypatch)
    arch = {"strategy": "spatial", "in_feat": 3, "normalization": norm, "num_classes": 52,
            "output_type": "logits",
            "st-gcn": {"in_feat": 3, "layers": 9, "kernel": 9, "importance": True,
                       "in_ch": [64, 64, 64, 64, 128, 128, 128, 256, 256],
                       "out_ch": [64, 64, 64, 128, 128, 128, 256, 256, 256],
                       "stride": [1, 1, 1, 2, 1, 1, 2, 1, 1], "residual": [1] * 9, "dropout": [0] * 9},
            "graph": P.PKU_MMD}
    torch.manual_seed(1538574472)
    m = P.MODELS["st-gcn"](rank=None, **arch)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randn(16, 3, 300, 25)
    ref = O.stgcn_model(x, sd, arch)
    m = m.to(DEV).set_compute_dtype("bf16")
    with torch.no_grad():
        y = m(x.to(DEV))
    torch.cuda.synchronize()
    assert len(calls) == (3 if norm == "LayerNorm" else 0)
    assert_close(y.float().cpu(), ref, 3e-2, "model logits (inference)")


def _ln_layer(P, seed, tcn_bias=None):
    torch.manual_seed(seed)
    layer = P.StgcnLayer(64, 64, (9, 25), 3, 25, stride=1, normalization="LayerNorm")
    if tcn_bias is not None:
        with torch.no_grad():
            layer.tcn[2].bias.copy_(tcn_bias)
    return layer


def test_fused_pack_cache_invalidation(P, monkeypatch):
    """The fused inference forward caches its packed weights (keyed by storage + in-place version):
    an optimizer-style in-place update is seen at once; a write through ``param.data`` (invisible to the
    version counter) is seen after train()/eval(), as documented (modules.StgcnLayer._drop_packs).  Each
    result equals the unfused route on the same weights."""
    calls = _count_fused(P, monkeypatch)
    A = _graph(P).to(DEV)
    layer = _ln_layer(P, 11).to(DEV).eval()
    P.set_compute_dtype(layer, "bf16")
    x = cl(torch.randn(4, 64, 40, 25), BF)

    def both():
        with torch.no_grad():
            y_f = layer(x, A)
            monkeypatch.setattr(P.routing.ROUTING, "fused_inference", False)
            y_u = layer(x, A)
            monkeypatch.setattr(P.routing.ROUTING, "fused_inference", True)
        torch.cuda.synchronize()
        return y_f.float(), y_u.float()

    y0, u0 = both()
    assert_close(y0, u0, 3e-2, "fused vs unfused")
    with torch.no_grad():  # optimizer-style in-place step: bumps the version counter
        layer.tcn[2].weight.mul_(-0.5)
        layer.gcn.conv.weight.add_(0.05)
    y1, u1 = both()
    assert (u1 - u0).abs().max() > 0.1
    assert_close(y1, u1, 3e-2, "after an in-place update")
    layer.tcn[2].weight.data.mul_(2.0)  # through .data: re-pack on eval()
    layer.eval()
    y2, u2 = both()
    assert (u2 - u1).abs().max() > 0.1
    assert_close(y2, u2, 3e-2, "after a .data write + eval()")
    assert len(calls) == 3


def test_fused_ln_large_bias(P):
    """LayerNorm statistics of z = tcn(...) + b with a large common bias (frame mean >> frame std): the
    fused kernel shifts its sums by the mean bias, so LN2 keeps fp32 precision (vs the fp32 oracle)."""
    A = _graph(P)
    g = torch.Generator().manual_seed(12)
    layer = _ln_layer(P, 12, tcn_bias=3000.0 + 0.5 * torch.randn(64, generator=g))
    sd = {k: v.clone() for k, v in layer.state_dict().items()}
    x = torch.randn(4, 64, 50, 25, generator=g)
    ref = O.stgcn_layer(x, A, sd, "", 9, 1, True, "LayerNorm")
    layer = layer.to(DEV).eval()
    P.set_compute_dtype(layer, "bf16")
    with torch.no_grad():
        y = layer(x.to(DEV), A.to(DEV))
    torch.cuda.synchronize()
    assert_close(y.float().cpu(), ref, 3e-2, "fused LN layer, bias 3000")


def test_fused_packs_follow_package_adam(P, monkeypatch):
    """The package's Adam writes parameters through raw pointers; it bumps their version counters, so a
    no_grad forward in train mode right after a step (no train()/eval() in between) repacks and equals the
    unfused route on the updated weights (stale fused packs)."""
    calls = _count_fused(P, monkeypatch)
    A = _graph(P).to(DEV)
    layer = _ln_layer(P, 13).to(DEV).train()
    P.set_compute_dtype(layer, "bf16")
    x = cl(torch.randn(4, 64, 40, 25), BF)
    with torch.no_grad():
        y0 = layer(x, A).float()
    opt = P.optim.Adam(layer.parameters(), lr=0.05)
    for p in layer.parameters():
        p.grad = torch.randn_like(p)
    v0 = [p._version for p in layer.parameters()]
    opt.step()
    assert all(p._version > v for p, v in zip(layer.parameters(), v0))
    with torch.no_grad():
        y1 = layer(x, A).float()
        monkeypatch.setattr(P.routing.ROUTING, "fused_inference", False)
        u1 = layer(x, A).float()
    torch.cuda.synchronize()
    assert (u1 - y0).abs().max() > 0.1
    assert_close(y1, u1, 3e-2, "fused forward after a package-Adam step")
    assert len(calls) == 2


def _spy_train(P, monkeypatch):
    calls = []
    orig = P.native.layer_fused

    def spy(*a, **k):
        calls.append(bool(k.get("train")))
        return orig(*a, **k)

    monkeypatch.setattr(P.native, "layer_fused", spy)
    return calls


@pytest.mark.parametrize("N,T,residual", [(3, 37, True), (2, 20, False), (64, 300, True)])
def test_ln_layer_fused_training(P, monkeypatch, N, T, residual):
    """Training forward of a LayerNorm 64 -> 64 stride-1 layer through the one-kernel layer (routing
    fused_ln_train), which also writes g, u and both LN statistics for the unfused backward: y and every
    gradient against the fp32 oracle (layernorm.py:22-28, stgcn.py:181-193; bf16 tolerance 4e-2 as the other
    bf16 layer tests) and against the unfused training route on the same inputs (2e-2); the fused kernel ran in
    training mode."""
    from conftest import assert_grad_close, grad_floor
    calls = _spy_train(P, monkeypatch)
    g = torch.Generator().manual_seed(21 + T)
    A = _graph(P)
    torch.manual_seed(21 + T)
    layer = P.StgcnLayer(64, 64, (9, 25), 3, 25, stride=1, residual=residual, normalization="LayerNorm")
    with torch.no_grad():  # non-trivial LayerNorm affines
        for nm in ("tcn.0", "tcn.3"):
            m = layer.get_submodule(nm)
            m.weight.copy_(1 + 0.2 * torch.randn(m.weight.shape, generator=g))
            m.bias.copy_(0.2 * torch.randn(m.bias.shape, generator=g))
    sd = {k: v.clone().requires_grad_(True) for k, v in layer.state_dict().items()}
    x = torch.randn(N, 64, T, 25, generator=g)
    dy = torch.randn(N, 64, T, 25, generator=g)
    small = N * T <= 200
    if small:
        xr = x.clone().requires_grad_(True)
        Ar = A.clone().requires_grad_(True)
        ref = O.stgcn_layer(xr, Ar, sd, "", 9, 1, residual, "LayerNorm")
        ref.backward(dy)
    layer = P.set_compute_dtype(layer.to(DEV), "bf16")
    out = {}
    for route in (True, False):
        monkeypatch.setattr(P.routing.ROUTING, "fused_ln_train", route)
        layer.zero_grad(set_to_none=True)
        xg = x.to(DEV).requires_grad_(True)
        Ag = A.to(DEV).requires_grad_(True)
        y = layer(xg, Ag)
        y.backward(dy.to(DEV))
        torch.cuda.synchronize()
        out[route] = (y.detach().float().cpu(), xg.grad.float().cpu(), Ag.grad.float().cpu(),
                      {k: p.grad.float().cpu() for k, p in layer.named_parameters()})
    assert calls == [True], calls  # the fused route ran once, in training mode; the unfused one not at all
    (yf, dxf, dAf, gf), (yu, dxu, dAu, gu) = out[True], out[False]
    # the two routes round differently (fused: g and LN1 statistics from the fp32 accumulators in one kernel;
    # unfused: LN1 statistics of the bf16-stored g), and ReLU masks flip where a pre-activation is within
    # rounding of 0: gradients are compared at the bf16 layer tolerance, as each route is against the oracle
    # (r04d: dx 4.3-6.3e-2 L2 apart at 0.7-0.8 % of elements beyond 2e-2, y 0.6e-2 apart)
    assert_close(yf, yu, 2e-2, "fused vs unfused y")
    assert_grad_close(dxf, dxu, 4e-2, "fused vs unfused dx")
    assert_grad_close(dAf, dAu, 4e-2, "fused vs unfused dA", reduction=True)
    for k in gu:
        assert_grad_close(gf[k], gu[k], 4e-2, f"fused vs unfused {k}", reduction=True)
    if small:
        tol = 4e-2
        assert_close(yf, ref, tol, "y")
        assert_grad_close(dxf, xr.grad, tol, "dx")
        assert_grad_close(dAf, Ar.grad, tol, "dA", reduction=True)
        grads = {k: v.grad for k, v in sd.items() if v.grad is not None}
        for k, gr in grads.items():
            assert_grad_close(gf[k], gr, tol, k, grad_floor(grads, k), reduction=True)


def test_ln_model_fused_training(P, monkeypatch):
    """ln/stgcn_vsc.json-style model (LayerNorm, Kt = 9, the config-2 widths, 9 layers) fwd + loss-free bwd in
    bf16 with the fused training route on its three 64 -> 64 layers: logits equal the unfused route's (2e-2) and
    the fp32 oracle's (3e-2), every parameter gradient the unfused route's at the bf16 layer tolerance (4e-2)."""
    from conftest import assert_grad_close
    calls = _spy_train(P, monkeypatch)
    arch = {"strategy": "spatial", "in_feat": 3, "normalization": "LayerNorm", "num_classes": 52,
            "output_type": "logits",
            "st-gcn": {"in_feat": 3, "layers": 9, "kernel": 9, "importance": True,
                       "in_ch": [64, 64, 64, 64, 128, 128, 128, 256, 256],
                       "out_ch": [64, 64, 64, 128, 128, 128, 256, 256, 256],
                       "stride": [1, 1, 1, 2, 1, 1, 2, 1, 1], "residual": [1] * 9, "dropout": [0] * 9}}
    torch.manual_seed(31)
    m = P.MODELS["st-gcn"](rank=None, **dict(arch, graph=P.PKU_MMD))
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randn(4, 3, 48, 25, generator=torch.Generator().manual_seed(32))
    with torch.no_grad():
        ref = O.stgcn_model(x, sd, dict(arch, graph=P.PKU_MMD))
    m = m.to(DEV).set_compute_dtype("bf16")
    out = {}
    for route in (True, False):
        monkeypatch.setattr(P.routing.ROUTING, "fused_ln_train", route)
        m.zero_grad(set_to_none=True)
        y = m(x.to(DEV))
        (y.float() ** 2).sum().backward()
        torch.cuda.synchronize()
        out[route] = (y.detach().float().cpu(), {k: p.grad.float().cpu() for k, p in m.named_parameters()})
    assert calls == [True] * 3, calls
    assert_close(out[True][0], ref, 3e-2, "fused-route logits vs oracle")
    assert_close(out[True][0], out[False][0], 2e-2, "fused vs unfused logits")
    for k, gu in out[False][1].items():
        assert_grad_close(out[True][1][k], gu, 4e-2, f"fused vs unfused {k}", reduction=True)

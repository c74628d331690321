"""AAGCN parity on the MI355X: attention adjacency (softmax(theta^T phi)) + per-sample-A ST-GCN layer,
against the reference's outputs (tests/golden/agcn_layer.npz, model_aagcn_bn_narrow.npz) and, at a
wider shape (ce = 16: vectorised attention path), against the CPU oracle."""
import pytest
import torch

from conftest import assert_close, assert_grad_close, bn_fed_bias, grad_floor, load_golden, sub
from oracle import stgcn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-3


@pytest.fixture(scope="module")
def P(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg


def test_agcn_layer_golden(P):
    from rtstgcn_amd.aagcn import AgcnLayer
    d = load_golden("agcn_layer")
    layer = AgcnLayer(16, 16, (9, 25), 3, 1, True, 0, 25, normalization="BatchNorm")
    layer.load_state_dict(sub(d, "sd/"), strict=True)
    layer = layer.to(DEV)
    x = d["x"].to(DEV).requires_grad_(True)
    y = layer(x, d["A"].to(DEV))
    assert_close(y, d["y"], TOL, "y")
    y.backward(d["dy"].to(DEV))
    assert_close(x.grad, d["dx"], TOL, "dx")
    grads = sub(d, "grad/")
    named = dict(layer.named_parameters())
    for k, g in grads.items():
        assert_close(named[k].grad, g, TOL, k, grad_floor(grads, k))


def test_aagcn_model_golden(P):
    d = load_golden("model_aagcn_bn_narrow")
    m = P.MODELS["aa-gcn"](rank=None, **d["arch"])
    m.load_state_dict(sub(d, "sd/"), strict=True)
    m = m.to(DEV)
    x = d["x"].to(DEV).requires_grad_(True)
    y = m(x)
    assert_close(y, d["y"], TOL, "y")
    y.backward(d["dy"].to(DEV))
    # 2 streams x 9 layers, softmax head: fp32 accumulation-order noise reaches ~1.3e-3 of max|dx| here
    assert_grad_close(x.grad, d["dx"], TOL, "dx")
    grads = sub(d, "grad/")
    named = dict(m.named_parameters())
    for k, g in grads.items():  # deepest grads (norm_in) carry the same accumulation-order noise
        assert_grad_close(named[k].grad, g, TOL, k, grad_floor(grads, k), reduction=True)


def test_agcn_layer_vs_oracle_c64(P):
    from rtstgcn_amd.aagcn import AgcnLayer
    torch.manual_seed(11)
    A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32)
    layer = AgcnLayer(64, 64, (9, 25), 3, 1, True, 0, 25, normalization="BatchNorm")
    with torch.no_grad():
        layer.B.copy_(0.05 * torch.randn(layer.B.shape))
    x = torch.randn(3, 64, 40, 25)
    sd = {k: v.clone().requires_grad_(True) for k, v in layer.state_dict().items()}
    xr = x.clone().requires_grad_(True)
    ref = O.agcn_layer(xr, A, sd, "", 9, 1, True, "BatchNorm", 3)
    dy = torch.randn(ref.shape)
    ref.backward(dy)
    layer = layer.to(DEV)
    xg = x.to(DEV).requires_grad_(True)
    y = layer(xg, A.to(DEV))
    y.backward(dy.to(DEV))
    assert_close(y, ref, TOL, "y")
    assert_grad_close(xg.grad, xr.grad, TOL, "dx")
    named = dict(layer.named_parameters())
    grads = {k: v.grad for k, v in sd.items() if v.grad is not None}
    for k, g in grads.items():
        assert_grad_close(named[k].grad, g, TOL, k, grad_floor(grads, k), reduction=True)


def test_aagcn_model_bit_reproducible(P):
    """Attention scores and per-sample dA reduce their T-chunk partials in a fixed order (no atomics):
    two identical fwd+bwd runs give bit-identical outputs and input gradients."""
    d = load_golden("model_aagcn_bn_narrow")
    m = P.MODELS["aa-gcn"](rank=None, **d["arch"])
    m.load_state_dict(sub(d, "sd/"), strict=True)
    m = m.to(DEV)
    outs = []
    for _ in range(2):
        x = d["x"].to(DEV).requires_grad_(True)
        y = m(x)
        y.backward(d["dy"].to(DEV))
        outs.append((y.detach().clone(), x.grad.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


AAGCN_ARCH = {"strategy": "spatial", "in_feat": 3, "output_type": "logits", "normalization": "BatchNorm",
              "num_classes": 52,
              "aa-gcn": {"layers": 9, "kernel": 9, "importance": True, "in_feat": 3,
                         "in_ch": [64, 64, 64, 64, 128, 128, 128, 256, 256],
                         "out_ch": [64, 64, 64, 128, 128, 128, 256, 256, 256],
                         "stride": [1, 1, 1, 2, 1, 1, 2, 1, 1], "residual": [1] * 9, "dropout": [0] * 9}}


@pytest.fixture(scope="module")
def aagcn_ref(P):
    """Config 5's model (as_is/aagcn_local.json: 2 streams, BN, 9 layers, config-2 channel schedule; B
    perturbed so the learnable adjacency term is exercised; output_type 'logits') and the oracle's fwd + bwd
    (oracle aagcn_model, reference aagcn.py:60-95,139-150) at N=16 T=300 in fp64 (the yardstick), fp32 and
    under bf16 autocast.  N=16: the temporal convs see 480 / 240 / 120 frame tiles, more than one per block
    of the persistent kernels at C = 64, 128.

    AAGCN is numerically sensitive: the attention softmax takes logits contracted over C'*T = 4800 terms, so
    relative input perturbations are amplified ~100x (the reference's own fp32 is ~2.6e-2 L2 from fp64 on dx
    here; its bf16 autocast is 9 % off on the logits and 100-400 % on the gradients)."""
    from test_gpu_bench_config import oracle_fwd_bwd
    torch.manual_seed(1538574472)
    arch = dict(AAGCN_ARCH, graph=P.PKU_MMD)
    m = P.MODELS["aa-gcn"](rank=None, **arch)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith(".B"):
                p.copy_(0.05 * torch.randn(p.shape))
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(16, 3, 300, 25, generator=gen)
    dy = torch.randn(16, 52, 1, generator=gen)
    far = P.Graph(**P.PKU_MMD).get_adjacency_raw()[2]
    fn = lambda xx, sd: O.aagcn_model(xx, sd, arch, far)  # noqa: E731
    refs = {"f64": oracle_fwd_bwd(fn, x, dy, sd0, torch.float64),
            "f32": oracle_fwd_bwd(fn, x, dy, sd0, torch.float32),
            "ac16": oracle_fwd_bwd(fn, x, dy, sd0, torch.float32, autocast_bf16=True)}
    return arch, sd0, x, dy, refs


@pytest.fixture(scope="module")
def aagcn_ref64(P):
    """Config 5 at its timed size, N = 64 T = 300: the same model and seeds as aagcn_ref, the oracle's fwd + bwd in
    fp64 (the yardstick) and fp32 (the reference's precision) on the CPU."""
    from test_gpu_bench_config import oracle_fwd_bwd
    torch.manual_seed(1538574472)
    arch = dict(AAGCN_ARCH, graph=P.PKU_MMD)
    m = P.MODELS["aa-gcn"](rank=None, **arch)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith(".B"):
                p.copy_(0.05 * torch.randn(p.shape))
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(64, 3, 300, 25, generator=gen)
    dy = torch.randn(64, 52, 1, generator=gen)
    far = P.Graph(**P.PKU_MMD).get_adjacency_raw()[2]
    fn = lambda xx, sd: O.aagcn_model(xx, sd, arch, far)  # noqa: E731
    refs = {"f64": oracle_fwd_bwd(fn, x, dy, sd0, torch.float64),
            "f32": oracle_fwd_bwd(fn, x, dy, sd0, torch.float32)}
    return arch, sd0, x, dy, refs


def _aagcn_run(P, arch, sd0, x, dy, dtype):
    m = P.MODELS["aa-gcn"](rank=None, **arch)
    m.load_state_dict(sd0, strict=True)
    m = m.to(DEV).set_compute_dtype(dtype)
    xg = x.to(DEV).requires_grad_(True)
    y = m(xg)
    y.backward(dy.to(DEV))
    got = {"logits": y.detach(), "dx": xg.grad}
    got.update({k: p.grad for k, p in m.named_parameters()})
    return {k: v.detach().double().cpu() for k, v in got.items()}


def _l2(t, ref):
    return ((t.double() - ref).norm() / ref.norm().clamp_min(1e-300)).item()


def _mx(t, ref):
    return ((t.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-300)).item()


def test_aagcn_model_fp32_n16_strict(P, aagcn_ref):
    """fp32 AAGCN (config-5 model) at N = 16, T = 300, held per tensor to the reference's own fp32: logits within the
    north_star 1e-3 of the reference's fp32, and EVERY gradient within 3x the reference's fp32 L2 error (vs fp64)
    + 1e-4.  A 1-2 % regression in any single fp32 kernel fails here (the N = 64 test below allows each tensor the
    model's 2 % fp32 noise floor at that size)."""
    arch, sd0, x, dy, refs = aagcn_ref
    r64, r32 = refs["f64"], refs["f32"]
    got = _aagcn_run(P, arch, sd0, x, dy, "fp32")
    assert_close(got["logits"], r32["logits"], 1e-3, "aagcn fp32 logits vs reference fp32")
    bad = []
    for k, ref in r64.items():
        print(f"[err] aagcn fp32 N=16 {k}: ours L2 {_l2(got[k], ref):.2e} | ref fp32 L2 {_l2(r32[k], ref):.2e}",
              flush=True)
        if bn_fed_bias(k) or k.endswith("phi.bias"):  # exact gradient 0 (phi's bias cancels in the softmax)
            continue
        if not torch.isfinite(got[k]).all() or _l2(got[k], ref) > 3 * _l2(r32[k], ref) + 1e-4:
            bad.append((k, f"{_l2(got[k], ref):.2e}", f"{_l2(r32[k], ref):.2e}"))
    assert not bad, f"fp32 AAGCN (N=16) further from fp64 than 3x the reference's fp32 on: {bad}"


def test_aagcn_model_fp32_config5(P, aagcn_ref64):
    """fp32 AAGCN at config 5's timed size (N = 64, T = 300): logits within the north_star 1e-3 of the
    reference's fp32; gradients as close to fp64 as the reference's fp32 on the median tensor (L2 ratio <= 1.5),
    and every tensor within 3x the reference's fp32 error + 0.02.  At N = 64 the model's own fp32 noise is at the
    2 % level (the reference's fp32 dx is 2.0e-2 L2 from fp64: the attention logits contract C'*T terms), so a
    single tensor's fp32 error depends on the summation order; the 0.02 floor is that noise level (r04c: our
    worst tensors 2.8e-2 / 1.5e-2 against the reference's 8.0e-3 / 4.8e-3, dx 2.15e-2 against 2.04e-2)."""
    arch, sd0, x, dy, refs = aagcn_ref64
    r64, r32 = refs["f64"], refs["f32"]
    got = _aagcn_run(P, arch, sd0, x, dy, "fp32")
    assert_close(got["logits"], r32["logits"], 1e-3, "aagcn fp32 logits vs reference fp32")
    bad, ratios = [], []
    for k, ref in r64.items():
        print(f"[err] aagcn fp32 {k}: ours L2 {_l2(got[k], ref):.2e} max {_mx(got[k], ref):.2e} | ref fp32 L2 "
              f"{_l2(r32[k], ref):.2e} max {_mx(r32[k], ref):.2e}", flush=True)
        if bn_fed_bias(k) or k.endswith("phi.bias"):  # exact gradient 0 (phi's bias cancels in the softmax)
            continue
        ratios.append(_l2(got[k], ref) / max(_l2(r32[k], ref), 1e-30))
        if not torch.isfinite(got[k]).all() or _l2(got[k], ref) > 3 * _l2(r32[k], ref) + 0.02:
            bad.append(k)
    ratios.sort()
    med = ratios[len(ratios) // 2]
    print(f"[err] aagcn fp32 L2 ratio ours / reference fp32: median {med:.3f}", flush=True)
    assert not bad and med <= 1.5, f"fp32 AAGCN vs fp64: bad {bad}, median ratio {med:.3f}"


def test_aagcn_model_bf16_config5(P, aagcn_ref):
    """Config 5's dtype (bf16) fwd + bwd vs fp64, beside the reference's own bf16 (autocast).  Ours keeps
    the attention branch in fp32 (aagcn.AgcnLayer.forward); the bf16 activations it reads still move the
    logits by a few %.  The gradients of this model are chaotic under ANY bf16 arithmetic: the reference's
    bf16 is 60-400 % L2 off fp64 on every weight, and single tensors swing with the rounding pattern — an
    A/B of two of our builds that agree to one bf16 ulp at kernel level (tools/ab_aagcn.py, seeds 0-2) put
    the worst tensor at 6.6x / 17.7x the truth's norm on one seed and the other way round on another.  So
    the gradients are checked as a distribution, not per tensor: finite everywhere; ours closer to fp64
    than the reference's bf16 on the median tensor (ratio <= 1); 90th-percentile ratio <= 3 (a systematic
    error would move the whole distribution).  The kernels themselves are pinned by
    test_aagcn_model_fp32_config5 and, in bf16 at these sizes, by test_gpu_bench_config's per-sample-A layer
    tests and test_gpu_kernels.test_amix.  Logits: max error within 1.5x of the reference's bf16 and
    cosine >= 0.99."""
    arch, sd0, x, dy, refs = aagcn_ref
    r64, r16 = refs["f64"], refs["ac16"]
    got = _aagcn_run(P, arch, sd0, x, dy, "bf16")
    bad, ratios = [], []
    for k, ref in r64.items():
        cos = torch.nn.functional.cosine_similarity(got[k].reshape(1, -1), ref.reshape(1, -1)).item()
        print(f"[err] aagcn bf16 {k}: ours L2 {_l2(got[k], ref):.2e} max {_mx(got[k], ref):.2e} cos {cos:.4f} | "
              f"ref bf16 L2 {_l2(r16[k], ref):.2e} max {_mx(r16[k], ref):.2e}", flush=True)
        if not torch.isfinite(got[k]).all():
            bad.append(k)
            continue
        if k == "logits":
            if _mx(got[k], ref) > 1.5 * _mx(r16[k], ref) or cos < 0.99:
                bad.append(k)
            continue
        if bn_fed_bias(k) or k.endswith("phi.bias"):
            continue
        ratios.append(_l2(got[k], ref) / max(_l2(r16[k], ref), 1e-30))
    ratios.sort()
    med, p90 = ratios[len(ratios) // 2], ratios[int(0.9 * len(ratios))]
    print(f"[err] aagcn bf16 L2 ratio ours / reference bf16: median {med:.3f}, p90 {p90:.3f}", flush=True)
    assert not bad and med <= 1.0 and p90 <= 3.0, f"bf16 AAGCN: bad {bad}, median {med:.3f}, p90 {p90:.3f}"


def test_aagcn_bf16_vs_fp32_per_tensor(P, aagcn_ref64):
    """Per tensor, config 5's bf16 path against the HIP fp32 path on the same inputs at N = 64.  The logits agree
    (cosine >= 0.99).  The gradients of this model are chaotic under ANY bf16 arithmetic (test_aagcn_model_bf16_
    config5: the reference's own bf16 autocast is 60-400 % L2 off fp64 on every weight; r04c measured our bf16
    vs fp32 cosines around 0 for dx), so per-tensor gradient cosines are printed as diagnostics and only
    finiteness is asserted; the bf16 gradients are judged against the reference's bf16 as a distribution in
    test_aagcn_model_bf16_config5, and per tensor in config 2 (test_model_bf16_vs_fp32_per_tensor)."""
    arch, sd0, x, dy, _ = aagcn_ref64
    g16 = _aagcn_run(P, arch, sd0, x, dy, "bf16")
    g32 = _aagcn_run(P, arch, sd0, x, dy, "fp32")
    bad, worst = [], (2.0, None)
    for k, ref in g32.items():
        if bn_fed_bias(k) or k.endswith("phi.bias"):
            continue
        cos = torch.nn.functional.cosine_similarity(g16[k].reshape(1, -1), ref.reshape(1, -1)).item()
        print(f"[err] aagcn bf16 vs fp32 {k}: cos {cos:.5f} L2 {_l2(g16[k], ref):.2e}", flush=True)
        worst = min(worst, (cos, k))
        if not torch.isfinite(g16[k]).all() or (k == "logits" and not cos >= 0.99):
            bad.append((k, round(cos, 4)))
    print(f"[err] aagcn bf16 vs fp32 worst cosine {worst[0]:.5f} ({worst[1]})", flush=True)
    assert not bad, f"bf16 AAGCN vs the HIP fp32 path: {bad}"


@pytest.mark.parametrize("cin,cout,stride,T", [(64, 64, 1, 300), (128, 256, 2, 150)])
def test_agcn_layer_bf16_vs_fp32_per_tensor(P, cin, cout, stride, T):
    """Per tensor where bf16 IS stable: one AgcnLayer at config-5 widths (N = 8), the bf16 path against the HIP fp32
    path on the same inputs, every gradient with cosine >= 0.98 (except the exact zeros: BN-fed conv biases, phi's
    bias).  A single layer does not amplify rounding the way the 9-layer 2-stream model does (fp64 with 2^-9 input
    noise: every gradient cosine >= 0.99 here, vs a median of 0.13 for the whole model,
    test_aagcn_sensitivity.py), so this pins the bf16 attention and per-sample-A kernels per tensor."""
    from rtstgcn_amd.aagcn import AgcnLayer
    torch.manual_seed(11)
    A = torch.tensor(P.Graph(**P.PKU_MMD).A, dtype=torch.float32)
    layer = AgcnLayer(cin, cout, (9, 25), 3, stride, True, 0, 25, normalization="BatchNorm")
    with torch.no_grad():
        layer.B.copy_(0.05 * torch.randn(layer.B.shape))
    x = torch.randn(8, cin, T, 25)
    dy = torch.randn(8, cout, (T - 1) // stride + 1, 25)
    sd0 = {k: v.clone() for k, v in layer.state_dict().items()}
    got = {}
    for dt in ("fp32", "bf16"):
        m = AgcnLayer(cin, cout, (9, 25), 3, stride, True, 0, 25, normalization="BatchNorm")
        m.load_state_dict(sd0, strict=True)
        m = P.set_compute_dtype(m.to(DEV), dt)
        xg = x.to(DEV).requires_grad_(True)
        y = m(xg, A.to(DEV))
        y.backward(dy.to(DEV, y.dtype).contiguous(memory_format=torch.channels_last))
        r = {"y": y.detach(), "dx": xg.grad}
        r.update({k: p.grad for k, p in m.named_parameters()})
        got[dt] = {k: v.detach().double().cpu() for k, v in r.items()}
    bad = []
    for k, ref in got["fp32"].items():
        if bn_fed_bias(k) or k.endswith("phi.bias"):
            continue
        cos = torch.nn.functional.cosine_similarity(got["bf16"][k].reshape(1, -1), ref.reshape(1, -1)).item()
        print(f"[err] agcn layer {cin}->{cout} bf16 vs fp32 {k}: cos {cos:.5f} L2 {_l2(got['bf16'][k], ref):.2e}",
              flush=True)
        if not cos >= 0.98:  # r05a: worst 0.9917 (phi.weight at 128 -> 256)
            bad.append((k, round(cos, 4)))
    assert not bad, f"bf16 AgcnLayer vs the HIP fp32 path: {bad}"

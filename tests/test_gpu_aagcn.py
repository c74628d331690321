"""AAGCN parity on the MI355X: attention adjacency (softmax(theta^T phi)) + per-sample-A ST-GCN layer,
against the reference's outputs (tests/golden/agcn_layer.npz, model_aagcn_bn_narrow.npz) and, at a
wider shape (ce = 16: vectorised attention path), against the CPU oracle."""
import pytest
import torch

from conftest import assert_close, assert_grad_close, grad_floor, load_golden, sub
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

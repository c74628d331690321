"""Window staging (window.hip): norm_in + fcn_in of WindowSegment's sliding windows
built from the padded capture without forming the windows, against the oracle applied to the
materialised windows (the reference's unfold, segment_generator.py:143; batchnorm.py:13-23 /
layernorm.py:22-28; stgcn.py:82-85).

* op level (layer_fn.WindowStageFunction): forward rows and the norm / fcn_in parameter gradients, both
  norms, fp32 (1e-4 forward, 1e-3 gradients) and bf16 (2e-2), window ranges that start inside the zero
  padding, mid-trial, short (nw < W) and the reference's segment size (1000 windows of W=50);
* model level: stgcn.Model on a WindowBatch == the oracle model on the materialised batch (fp32, fwd and
  every parameter gradient), both norms; and == the same HIP model fed the materialised tensor.
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import assert_close, assert_grad_close, bn_fed_bias
from oracle import stgcn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def P(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg


def _norm_params(mode, C, V, g):
    if mode == 0:
        return 1 + 0.3 * torch.randn(V * C, generator=g), 0.2 * torch.randn(V * C, generator=g)
    return 1 + 0.3 * torch.randn(C, 1, V, generator=g), 0.2 * torch.randn(C, 1, V, generator=g)


def _oracle_stage(win, mode, nw_, nb_, w, b):
    xn = O.input_batchnorm(win, nw_, nb_) if mode == 0 else O.layernorm_cv(win, nw_, nb_)
    return F.conv2d(xn, w, b)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("L,W,n0,nw,dt", [(37, 5, 0, 20, "fp32"), (300, 50, 100, 200, "fp32"), (61, 9, 7, 3, "fp32"),
                                          (1100, 50, 0, 1000, "bf16"), (400, 50, 37, 300, "fp32")])
def test_window_stage_op(P, mode, L, W, n0, nw, dt):
    g = torch.Generator().manual_seed(L + W + n0 + mode)
    C, V, Cout = 3, 25, 64
    dtype = torch.float32 if dt == "fp32" else torch.bfloat16
    cap = torch.randn(1, C, L, V, generator=g) * 0.7 + 0.2
    padded = F.pad(cap, (0, 0, W - 1, 0))
    nw_, nb_ = _norm_params(mode, C, V, g)
    w = torch.randn(Cout, C, 1, 1, generator=g) / 3 ** 0.5
    b = 0.1 * torch.randn(Cout, generator=g)
    batch = P.segment.WindowBatch(padded, n0, nw, W)
    win = batch.materialize()
    refp = [t.clone().requires_grad_(True) for t in (nw_, nb_, w, b)]
    ref = _oracle_stage(win, mode, *refp)
    G = torch.randn(ref.shape, generator=g)
    if dtype == torch.bfloat16:
        G = G.to(torch.bfloat16).float()
    ref.backward(G)

    hp = [t.to(DEV).requires_grad_(True) for t in (nw_, nb_, w, b)]
    y = P.layer_fn.WindowStageFunction.apply(padded.to(DEV), n0, nw, W, *hp, mode, dtype)
    assert y.shape == (nw, Cout, W, V) and y.dtype == dtype
    tol = 1e-4 if dt == "fp32" else 2e-2
    assert_close(y.float(), ref, tol, "staged rows")
    y.backward(G.to(DEV, dtype).contiguous(memory_format=torch.channels_last))
    gtol = 1e-3 if dt == "fp32" else 2e-2
    for name, h, r in zip(("norm.weight", "norm.bias", "fcn_in.weight", "fcn_in.bias"), hp, refp):
        assert_grad_close(h.grad, r.grad, gtol, name, reduction=True)


ARCH = {"strategy": "spatial", "in_feat": 3, "num_classes": 7, "output_type": "logits",
        "st-gcn": {"in_feat": 3, "layers": 2, "kernel": 9, "importance": True, "in_ch": [64, 64], "out_ch": [64, 64],
                   "stride": [1, 1], "residual": [1, 1], "dropout": [0, 0]}}


@pytest.mark.parametrize("norm", ["BatchNorm", "LayerNorm"])
def test_model_on_window_batch(P, norm):
    arch = dict(ARCH, normalization=norm, graph=P.PKU_MMD)
    torch.manual_seed(11)
    m = P.MODELS["st-gcn"](rank=None, **arch)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(4)
    for k in sd:
        if k.startswith("norm_in") or k.startswith("fcn_in"):
            sd[k] = sd[k] + 0.2 * torch.randn(sd[k].shape, generator=g)
    m.load_state_dict(sd)
    L, W = 90, 20
    cap = torch.randn(1, 3, L, 25, generator=g)
    seg = P.segment.WindowSegment(world_size=1, rank=DEV, stages=1, num_classes=7, graph={"num_node": 25},
                                  in_feat=3, receptive_field=W, segment=40)
    ps, pe = seg.pad_sequence(L)
    padded = F.pad(cap, (0, 0, ps, pe)).to(DEV)
    labels = torch.zeros(1, L, dtype=torch.long, device=DEV)
    batches = [b for b, _, _ in seg.get_segment(padded, labels)]
    assert len(batches) == 2 and batches[1].n0 == 39  # the second segment starts one window early
    xb = batches[1]
    win = xb.materialize().cpu()

    rsd = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and k != "A" else v) for k, v in sd.items()}
    ref = O.stgcn_model(win, rsd, arch)
    G = torch.randn(ref.shape, generator=g)
    ref.backward(G)

    m = m.to(DEV)
    y = m(xb)
    assert_close(y, ref, 1e-3, "logits (staged)")
    y.backward(G.to(DEV))
    for k, p in m.named_parameters():
        if norm == "BatchNorm" and bn_fed_bias(k):  # exact gradient 0 (BN cancels it): bound by the weight grad
            assert p.grad.abs().max().item() <= 1e-4 * rsd[k[:-4] + "weight"].grad.abs().max().item(), k
            continue
        assert_grad_close(p.grad, rsd[k].grad, 1e-3, k, reduction=True)

    m.zero_grad()
    y2 = m(xb.materialize())  # the same HIP model on the reference's materialised tensor
    assert_close(y, y2, 1e-4, "staged vs materialised")


def test_aagcn_on_window_batch(P):
    """aa-gcn (both streams; the bone stream's windows are the windows of the capture's bones): staged ==
    the same HIP model on the materialised batch, logits and every parameter gradient (fp32)."""
    arch = {"strategy": "spatial", "in_feat": 3, "num_classes": 7, "output_type": "logits",
            "normalization": "BatchNorm", "graph": P.PKU_MMD,
            "aa-gcn": {"in_feat": 3, "layers": 2, "kernel": 9, "importance": True, "in_ch": [64, 64],
                       "out_ch": [64, 64], "stride": [1, 1], "residual": [1, 1], "dropout": [0, 0]}}
    torch.manual_seed(5)
    m = P.MODELS["aa-gcn"](rank=None, **arch).to(DEV)
    g = torch.Generator().manual_seed(6)
    padded = F.pad(torch.randn(1, 3, 60, 25, generator=g), (0, 0, 19, 0)).to(DEV)
    xb = P.segment.WindowBatch(padded, 3, 30, 20)
    G = torch.randn(30, 7, generator=g).to(DEV)
    y = m(xb)
    (y.reshape(30, 7) * G).sum().backward()
    grads = {k: p.grad.clone() for k, p in m.named_parameters()}
    m.zero_grad()
    y2 = m(xb.materialize())
    (y2.reshape(30, 7) * G).sum().backward()
    assert_close(y, y2, 1e-4, "aagcn logits staged vs materialised")
    for k, p in m.named_parameters():
        if bn_fed_bias(k) or k.endswith("phi.bias"):
            continue
        assert_grad_close(grads[k], p.grad, 1e-3, k, reduction=True)

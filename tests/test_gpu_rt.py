"""RT-ST-GCN parity on the MI355X against the reference's own outputs (tests/golden/rt_*.npz):
offline (training) model fwd + bwd, and the per-frame online model (FIFO state on device).
Stride 1: offline == online in the reference; reference strides (layers 3, 6 at stride 2): each form
matches its own reference form (the reference's two forms diverge)."""
import pytest
import torch

from conftest import assert_close, grad_floor, load_golden, sub

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-3


@pytest.fixture(scope="module")
def P(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg


@pytest.mark.parametrize("case", ["stride1", "ref_strides"])
def test_rt_offline_golden(P, case):
    d = load_golden("rt_" + case)
    m = P.MODELS["rt-st-gcn"](rank=None, **d["arch"])
    m.load_state_dict(sub(d, "sd/"), strict=True)
    m = m.to(DEV)
    x = d["x"].to(DEV).requires_grad_(True)
    y = m(x)
    assert_close(y, d["y_offline"], TOL, "offline y")
    y.backward(d["dy"].to(DEV))
    assert_close(x.grad, d["dx"], TOL, "offline dx")
    grads = sub(d, "grad/")
    named = dict(m.named_parameters())
    for k, g in grads.items():
        assert_close(named[k].grad, g, TOL, k, grad_floor(grads, k))


@pytest.mark.parametrize("case", ["stride1", "ref_strides"])
def test_rt_online_golden(P, case):
    d = load_golden("rt_" + case)
    m = P.MODELS["rt-st-gcn"](rank=None, **d["arch"])
    m.load_state_dict(sub(d, "sd/"), strict=True)
    m = m.to(DEV).eval()
    m.prepare_benchmark({})
    x = d["x"].to(DEV)
    with torch.no_grad():
        outs = [m(x[:, :, i:i + 1]) for i in range(x.shape[2])]
    y = torch.cat(outs, dim=2)
    assert_close(y, d["y_online"], TOL, "online y")
    # state reset reproduces the stream from scratch
    m.reset_state()
    with torch.no_grad():
        y2 = torch.cat([m(x[:, :, i:i + 1]) for i in range(x.shape[2])], dim=2)
    assert_close(y2, y, 1e-6, "online after reset")

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


@pytest.fixture(params=["one_launch", "per_layer"])
def rt_route(request, pkg):
    """Both per-frame routes: the whole frame as one persistent launch (stgcn_rt_frame, default) and the
    two-launches-per-layer form (routing.rt_one_launch off)."""
    R = pkg.routing.ROUTING
    prev = R.rt_one_launch
    R.rt_one_launch = request.param == "one_launch"
    yield request.param
    R.rt_one_launch = prev


def _frame_status_ok(m, route):
    """The one-launch kernel's barrier never gave up (its bounded spin sets the status word)."""
    if route == "one_launch":
        st = getattr(m, "_frame_status", None)
        assert st is not None, "the one-launch route did not run"
        assert int(st.item()) == 0, "stgcn_rt_frame: a grid-barrier wait gave up"


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
def test_rt_online_golden(P, case, rt_route):
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
    _frame_status_ok(m, rt_route)


CONFIG3_LAYERS = {"layers": 9, "kernel": 9, "in_ch": [64, 64, 64, 64, 128, 128, 128, 256, 256],
                  "out_ch": [64, 64, 64, 128, 128, 128, 256, 256, 256], "residual": [1] * 9, "dropout": [0.0] * 9,
                  "latency": False, "importance": True, "in_feat": 3, "buffer": 1, "stages": 1}


@pytest.mark.parametrize("strides", [[1] * 9, [1, 1, 1, 2, 1, 1, 2, 1, 1]], ids=["stride1", "ref_strides"])
def test_rt_online_config3_widths(P, strides, rt_route):
    """Config 3 at its own widths (config/pku-mmd/ln/rtstgcn_local.json: LayerNorm, K = 9, 64 -> 256 channels,
    V*C up to 6 400): the per-frame kernels (rt_fused.hip; rt_norm's several values per thread, rt_gcn at
    Cin 64-256) over 48 frames (> every FIFO: 17 frames at stride 2), eager and replayed as a HIP graph, vs
    the oracle's online form (rtstgcn.py:528-553, 591-627), fp32 1e-3."""
    from oracle import stgcn_oracle as O
    arch = {"strategy": "spatial", "in_feat": 3, "stages": 1, "kernel": 9, "output_type": "logits",
            "normalization": "LayerNorm", "segment": 500, "num_classes": 52,
            "rt-st-gcn": dict(CONFIG3_LAYERS, stride=strides), "graph": P.PKU_MMD}
    torch.manual_seed(21)
    m = P.MODELS["rt-st-gcn"](rank=None, **arch)
    sd = m.state_dict()
    g = torch.Generator().manual_seed(22)
    for k in sd:  # non-trivial norms, biases and edge importance
        if "edge_importance" in k:
            sd[k] = 1 + 0.1 * torch.randn(sd[k].shape, generator=g)
        elif ("bn_relu" in k or "residual.1" in k or "norm_in" in k) and k.endswith("weight"):
            sd[k] = 1 + 0.2 * torch.randn(sd[k].shape, generator=g)
        elif k.endswith("bias"):
            sd[k] = 0.1 * torch.randn(sd[k].shape, generator=g)
    m.load_state_dict(sd, strict=True)
    F_ = 48
    x = torch.randn(1, 3, F_, 25, generator=g)
    with torch.no_grad():
        ref = O.rt_model_online(x, {k: v.clone() for k, v in sd.items()}, arch)
    m = m.to(DEV).eval()
    m.prepare_benchmark(arch)
    xd = x.to(DEV)
    with torch.no_grad():
        y = torch.cat([m(xd[:, :, i:i + 1]) for i in range(F_)], dim=2)
    torch.cuda.synchronize()
    assert_close(y, ref, TOL, f"config-3 online eager {strides} {rt_route}")
    # the same stream replayed as a HIP graph of one per-frame step (FIFO state on the device)
    m.reset_state()
    x_static = torch.zeros_like(xd[:, :, :1])
    with torch.no_grad():
        for i in range(3):
            x_static.copy_(xd[:, :, i:i + 1])
            m(x_static)
        m.reset_state()
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph):
                y_static = m(x_static)
        torch.cuda.current_stream().wait_stream(s)
        m.reset_state()
        outs = []
        for i in range(F_):
            x_static.copy_(xd[:, :, i:i + 1])
            graph.replay()
            outs.append(y_static.clone())
    torch.cuda.synchronize()
    assert_close(torch.cat(outs, dim=2), ref, TOL, f"config-3 online graph {strides} {rt_route}")
    _frame_status_ok(m, rt_route)


@pytest.mark.parametrize("blocks", [1, 3, 64, 200])
def test_rt_frame_block_counts(P, blocks):
    """stgcn_rt_frame at several workgroup counts (1: no cross-workgroup hand-off at all; 3: several channel pairs
    per workgroup; 200: idle workgroups that only take part in the barriers) gives the same frames as the
    two-launches-per-layer route, over 12 frames of config 3's widths (the FIFOs wrap), at fp32 rounding."""
    R = P.routing.ROUTING
    arch = {"strategy": "spatial", "in_feat": 3, "stages": 1, "kernel": 9, "output_type": "logits",
            "normalization": "LayerNorm", "segment": 500, "num_classes": 52,
            "rt-st-gcn": dict(CONFIG3_LAYERS, stride=[1, 1, 1, 2, 1, 1, 2, 1, 1]), "graph": P.PKU_MMD}
    torch.manual_seed(5)
    m = P.MODELS["rt-st-gcn"](rank=None, **arch).to(DEV).eval()
    m.prepare_benchmark(arch)
    x = torch.randn(1, 3, 12, 25, device=DEV)
    prev = R.rt_one_launch
    try:
        R.rt_one_launch = False
        with torch.no_grad():
            ref = torch.cat([m(x[:, :, i:i + 1]) for i in range(12)], dim=2)
        m.reset_state()
        R.rt_one_launch = True
        m._frame_pack = None
        with torch.no_grad():
            m(x[:, :, :1])  # builds the descriptor
            m.reset_state()
            m._frame_pack[1][0].blocks = blocks
            y = torch.cat([m(x[:, :, i:i + 1]) for i in range(12)], dim=2)
    finally:
        R.rt_one_launch = prev
    torch.cuda.synchronize()
    assert int(m._frame_status.item()) == 0
    assert_close(y, ref, 1e-4, f"rt_frame blocks={blocks}")

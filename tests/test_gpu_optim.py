"""optim.Adam (csrc/adam.hip: every parameter of a group in one launch) against torch.optim.Adam — the
reference's optimizer (processor.py:579, stepped at processor.py:561) — on the same parameters and gradients:
sizes below / across / far above one 2048-element block and not multiples of 4, a parameter without a gradient
(skipped, its step count unchanged, as torch does), a non-contiguous gradient, weight decay, several steps;
the state_dict round trip in both directions; and the config-2 model's parameters through one training step."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def P(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(3,), (64,), (2048,), (2049,), (5, 7, 11), (256, 256, 9, 1), (75,), (1,)]
    return [torch.randn(s, generator=g).to(DEV) for s in shapes]


def _grads(params, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(p.shape, generator=g).to(DEV) for p in params]


# the kernel follows the default (foreach) implementation's operations in fp32; fused-vs-foreach style reordering
# would show at ~1e-6
TOL = dict(rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_adam_matches_torch(P, wd):
    ref = [p.clone().requires_grad_(True) for p in _params(0)]
    got = [p.clone().requires_grad_(True) for p in _params(0)]
    o_ref = torch.optim.Adam(ref, lr=5e-4, weight_decay=wd)
    o_got = P.optim.Adam(got, lr=5e-4, weight_decay=wd)
    for it in range(6):
        gs = _grads(ref, 10 + it)
        for k, (a, b, g) in enumerate(zip(ref, got, gs)):
            if k == 1 and it in (2, 3):  # no gradient this step: skipped, step count not advanced
                a.grad = b.grad = None
                continue
            a.grad = g.clone()
            # k == 4: a non-contiguous gradient of the right shape
            b.grad = g.clone() if k != 4 else g.transpose(0, 2).contiguous().transpose(0, 2)
        o_ref.step()
        o_got.step()
        torch.cuda.synchronize()
        for k, (a, b) in enumerate(zip(ref, got)):
            torch.testing.assert_close(b.detach(), a.detach(), **TOL, msg=lambda m: f"step {it} param {k}: {m}")
            sa, sb = o_ref.state[a], o_got.state[b]
            assert float(sb["step"]) == float(sa["step"]), (it, k)
            torch.testing.assert_close(sb["exp_avg"], sa["exp_avg"], **TOL)
            torch.testing.assert_close(sb["exp_avg_sq"], sa["exp_avg_sq"], **TOL)


def test_adam_state_dict_round_trip(P):
    ref = [p.clone().requires_grad_(True) for p in _params(1)]
    got = [p.clone().requires_grad_(True) for p in _params(1)]
    o_ref = torch.optim.Adam(ref, lr=1e-3)
    for it in range(3):
        for a, g in zip(ref, _grads(ref, 20 + it)):
            a.grad = g
        o_ref.step()
    with torch.no_grad():
        for a, b in zip(ref, got):
            b.copy_(a)
    o_got = P.optim.Adam(got, lr=1e-3)
    o_got.load_state_dict(o_ref.state_dict())  # torch -> package
    for it in range(2):
        gs = _grads(ref, 30 + it)
        for a, b, g in zip(ref, got, gs):
            a.grad, b.grad = g.clone(), g.clone()
        o_ref.step()
        o_got.step()
    for a, b in zip(ref, got):
        torch.testing.assert_close(b.detach(), a.detach(), **TOL)
    back = torch.optim.Adam([p.detach().clone() for p in got], lr=1e-3)
    back.load_state_dict(o_got.state_dict())  # package -> torch
    for pa, pb in zip(o_got.param_groups[0]["params"], back.param_groups[0]["params"]):
        sa, sb = o_got.state[pa], back.state[pb]
        assert float(sa["step"]) == float(sb["step"]) == 5.0
        torch.testing.assert_close(sb["exp_avg"], sa["exp_avg"], rtol=0, atol=0)


def test_adam_model_step(P):
    """The config-2 model's 96 parameters (bench.py's optimizer) after one training step: same update as torch."""
    import bench
    torch.manual_seed(5)
    m = P.MODELS["st-gcn"](rank=None, **dict(bench.ARCH, graph=P.PKU_MMD)).to(DEV)
    params = [p for p in m.parameters() if p.requires_grad]
    g = torch.Generator().manual_seed(6)
    for p in params:
        p.grad = torch.randn(p.shape, generator=g).to(DEV)
    ref = [p.detach().clone().requires_grad_(True) for p in params]
    for a, p in zip(ref, params):
        a.grad = p.grad.clone()
    o_ref = torch.optim.Adam(ref, lr=5e-4)
    o_got = P.optim.Adam(params, lr=5e-4)
    assert len(params) <= 256
    for _ in range(2):
        o_ref.step()
        o_got.step()
    for a, p in zip(ref, params):
        torch.testing.assert_close(p.detach(), a.detach(), **TOL)


def test_adam_graph_replay(P):
    """optim.Adam captured in a HIP graph (as parallel.GraphedStep / bench.py --graph capture it): replaying the
    captured step with new gradients copied into the same .grad tensors gives bit-identical parameters, moments
    and step counts to eager steps (device step counters; gradient pointers baked into the captured launch)."""
    ref = [p.clone().requires_grad_(True) for p in _params(2)]
    got = [p.clone().requires_grad_(True) for p in _params(2)]
    o_ref = P.optim.Adam(ref, lr=1e-3)
    o_got = P.optim.Adam(got, lr=1e-3)
    grads = [_grads(ref, 40 + it) for it in range(4)]
    for a, b, g in zip(ref, got, grads[0]):  # first step eager on both (allocates the flat state)
        a.grad, b.grad = g.clone(), g.clone()
    o_ref.step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        o_got.step()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            o_got.step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    # capture does not execute: one eager step so far on both
    for it in range(1, 4):
        for a, b, g in zip(ref, got, grads[it]):
            a.grad.copy_(g)
            b.grad.copy_(g)
        o_ref.step()
        graph.replay()
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(a.detach(), b.detach())
        assert torch.equal(o_ref.state[a]["exp_avg_sq"], o_got.state[b]["exp_avg_sq"])
        assert float(o_ref.state[a]["step"]) == float(o_got.state[b]["step"]) == 4.0


def test_adam_many_tensors(P):
    """More tensors than one launch carries (STGCN_ADAM_MAXT = 256; the AAGCN 2-stream model has more): the
    group is split into launches, same update as torch."""
    g0 = torch.Generator().manual_seed(11)
    shapes = [(int(torch.randint(1, 300, (1,), generator=g0)),) for _ in range(300)]
    base = [torch.randn(s, generator=g0).to(DEV) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in base]
    got = [p.clone().requires_grad_(True) for p in base]
    o_ref, o_got = torch.optim.Adam(ref, lr=5e-4), P.optim.Adam(got, lr=5e-4)
    for it in range(3):
        for a, b in zip(ref, got):
            g = torch.randn(a.shape, generator=g0).to(DEV)
            a.grad, b.grad = g.clone(), g.clone()
        o_ref.step()
        o_got.step()
    for a, b in zip(ref, got):
        torch.testing.assert_close(b.detach(), a.detach(), **TOL)
        assert float(o_got.state[b]["step"]) == 3.0


def test_graphed_step_skips_unused_params(P):
    """parallel.GraphedStep with a parameter that gets no gradient (weight decay on): replays leave it and its
    Adam state untouched, as eager torch.optim.Adam steps do, and train the others exactly like eager steps."""
    g0 = torch.Generator().manual_seed(5)
    w0 = torch.randn(16, 8, generator=g0).to(DEV)
    u0 = torch.randn(8, generator=g0).to(DEV)
    xs = [torch.randn(4, 16, generator=g0).to(DEV) for _ in range(4)]

    def make():
        w = w0.clone().requires_grad_(True)
        unused = u0.clone().requires_grad_(True)
        return w, unused

    w_ref, u_ref = make()
    o_ref = torch.optim.Adam([w_ref, u_ref], lr=1e-2, weight_decay=0.1)
    for x in xs:
        o_ref.zero_grad()
        (x @ w_ref).square().sum().backward()
        o_ref.step()
    w, u = make()
    o = P.optim.Adam([w, u], lr=1e-2, weight_decay=0.1)
    xin = xs[0].clone()
    gstep = P.parallel.GraphedStep(lambda: (xin @ w).square().sum(), [w, u], o)  # runs xs[0] eagerly
    for x in xs[1:]:
        xin.copy_(x)
        gstep()
    torch.cuda.synchronize()
    assert u.grad is None and torch.equal(u.detach(), u0)
    assert u not in o.state or float(o.state[u]["step"]) == 0.0
    torch.testing.assert_close(w.detach(), w_ref.detach(), **TOL)

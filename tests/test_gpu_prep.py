"""One-launch weight preparation (native.PrepPlan / prep.hip, stgcn.Model._prepared): every pack the model's
layers read in a training step equals, bit for bit, the single-job launch it replaces (pack_weight,
pack_weight_frag / _s2frag, gconv_weights_bias, gconv_weights trans) on the product A * M the model feeds
the layer; and a training step through the plan gives bit-identical outputs and gradients to one that packs
per call (routing.prep_plan off; fp32 weight gradients up to the atomics' summation order)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def P(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg


def _model(P, dtype):
    import bench
    torch.manual_seed(3)
    m = P.MODELS["st-gcn"](rank=None, **dict(bench.ARCH, graph=P.PKU_MMD))
    g = torch.Generator().manual_seed(4)
    with torch.no_grad():
        for p in m.edge_importance:
            p.add_(0.1 * torch.randn(p.shape, generator=g))
        for name, p in m.named_parameters():
            if name.endswith("bias"):
                p.add_(0.1 * torch.randn(p.shape, generator=g))
    return m.to(DEV).set_compute_dtype(dtype)


def _buf(t):
    """The whole allocation behind a pack (plain pack + fragment image)."""
    return t._base if t._base is not None else t


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_plan_packs_equal_single_launches(P, dtype):
    K = P.native
    m = _model(P, dtype)
    dt = m.compute_dtype
    plan = m._prepared()
    torch.cuda.synchronize()
    assert plan is not None and plan.nblocks > 0
    for i, gcn in enumerate(m.gcn_networks):
        pk = plan.layers[i]
        Ai = (m.A * m.edge_importance[i]).detach()
        sup = gcn._gsup
        P_, Cout, Cin = Ai.shape[0], gcn.tcn[2].out_channels, gcn.gcn.conv.in_channels
        wg2 = gcn.gcn.conv.weight.detach().reshape(P_ * Cout, Cin).contiguous()
        w, b2 = K.gconv_weights(Ai, wg2, sup, Cout, Cin, False, dt, bias=gcn.gcn.conv.bias.detach())
        # slots j >= deg[joint] are never written (nor read by gconv): compare the used ones
        used = (torch.arange(sup.J, device=DEV)[None, :] < sup.deg[:, None])
        assert torch.equal(pk.gw[0][used], w[used]) and torch.equal(pk.gw[1], b2), f"layer {i} graph-conv weights"
        if pk.gwT is not None:
            usedT = (torch.arange(sup.J, device=DEV)[None, :] < sup.rdeg[:, None])
            wT = K.gconv_weights(Ai, wg2, sup, Cout, Cin, True, dt)
            assert torch.equal(pk.gwT[usedT], wT[usedT]), f"layer {i} transposed"
        wt = gcn.tcn[2].weight.detach().squeeze(-1)
        ref = K.pack_weight(wt.permute(2, 0, 1), dt, stride=gcn.stride)[0]
        assert torch.equal(_buf(pk.wt[0]), _buf(ref)), f"layer {i} temporal pack"
        ref = K.pack_weight(wt.permute(2, 1, 0), dt, stride=gcn.stride, trans=True)[0]
        assert torch.equal(_buf(pk.wtT[0]), _buf(ref)), f"layer {i} temporal data-grad pack"
        if gcn.is_residual_conv:
            wr = gcn.residual[0].weight.detach().view(Cout, Cin)
            assert torch.equal(_buf(pk.wr[0]), _buf(K.pack_weight(wr.unsqueeze(0), dt)[0]))
            assert torch.equal(_buf(pk.wrT[0]), _buf(K.pack_weight(wr.t().unsqueeze(0), dt)[0]))


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_plan_step_bit_identical(P, monkeypatch, dtype):
    torch.manual_seed(7)
    x = torch.randn(4, 3, 64, 25, device=DEV)
    dy = torch.randn(4, 52, 1, device=DEV)
    out = {}
    for on in (True, False):
        monkeypatch.setattr(P.routing.ROUTING, "prep_plan", on)
        m = _model(P, dtype)
        y = m(x)
        y.backward(dy)
        torch.cuda.synchronize()
        out[on] = (y.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()})
        assert (m._plan is not None) == on
    assert torch.equal(out[True][0], out[False][0])
    for k, g in out[True][1].items():
        if dtype == "fp32":
            # fp32 weight gradients run on the generic kernels with fp32 atomics (conv_wgrad.hip): equal up to
            # summation order (bf16 below is bit-exact end to end)
            torch.testing.assert_close(g, out[False][1][k], rtol=1e-5, atol=1e-6)
            continue
        assert torch.equal(g, out[False][1][k]), k

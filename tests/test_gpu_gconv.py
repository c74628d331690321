"""Joint-gathered graph conv (gconv.hip) vs the reference's conv1x1 -> einsum(A) formulation
(models/utils/tgcn.py:71-79) in plain PyTorch fp32: forward, data grad, weight and adjacency grads."""
import pytest
import torch
import torch.nn.functional as F

from conftest import assert_close

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def K(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg.native


def cl(x, dtype=torch.float32):
    return x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)


def ref_gcn(x, A, W, b):
    P, V = A.shape[0], A.shape[-1]
    y = F.conv2d(x, W.view(W.shape[0], -1, 1, 1), b)
    n, kc, t, v = y.shape
    return torch.einsum("nkctv,kvw->nctw", y.view(n, P, kc // P, t, v), A)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("Cin,Cout,N,T", [(64, 64, 3, 37), (128, 256, 2, 19), (8, 64, 2, 11), (256, 128, 2, 7),
                                          (24, 40, 3, 5), (256, 256, 2, 9)])
def test_gconv_fwd_bwd(K, pkg, dtype, tol, Cin, Cout, N, T):
    torch.manual_seed(3)
    A0 = torch.tensor(pkg.Graph(**pkg.PKU_MMD).A, dtype=torch.float32)
    imp = torch.rand(A0.shape) + 0.5
    A = (A0 * imp).requires_grad_(True)
    P, V = A.shape[0], A.shape[-1]
    x = torch.randn(N, Cin, T, V, requires_grad=True)
    W = (torch.randn(P * Cout, Cin) / Cin ** 0.5).requires_grad_(True)
    b = torch.randn(P * Cout)
    ref = ref_gcn(x, A, W, torch.zeros_like(b))
    dy = torch.randn(ref.shape)
    ref.backward(dy)

    sup = K.GraphSupport(A0.to(DEV))
    Ad, Wd = A.detach().to(DEV).contiguous(), W.detach().to(DEV).contiguous()
    wpk = K.gconv_weights(Ad, Wd, sup, Cout, Cin, False, dtype)
    bias2d = K.gcn_bias(Ad, b.to(DEV), N, Cout)
    st = torch.zeros((K.gconv_row_blocks(N * T, V), wpk.shape[2], 4), device=DEV)
    g = K.gconv(cl(x.detach(), dtype), wpk, sup, Cin, Cout, bias=bias2d, stats=st)
    ref_b = ref_gcn(x.detach(), A.detach(), W.detach(), b)
    assert_close(g.float(), ref_b, tol, "gconv fwd")
    mr, _, _ = K.bn_finalize(st, st.shape[0], wpk.shape[2], Cout, None, None)
    assert_close(mr[:, 0].cpu(), ref_b.mean(dim=(0, 2, 3)), 1e-4 if dtype == torch.float32 else 2e-3, "stats mean")

    wT = K.gconv_weights(Ad, Wd, sup, Cout, Cin, True, dtype)
    dx = K.gconv(cl(dy, dtype), wT, sup, Cout, Cin, trans=True)
    assert_close(dx.float(), x.grad, tol, "gconv dgrad")
    rs_ok = K.gconv_wgrad_rowsum_ok(sup, Cin, Cout, dtype)
    rowsum = torch.empty((V, Cout), device=DEV) if rs_ok else None
    dweff = K.gconv_wgrad(cl(x.detach(), dtype), cl(dy, dtype), sup, Cin, Cout, rowsum=rowsum)
    if rs_ok:  # per-joint row sums of dy (the bias-through-A gradient), fused into the same kernel
        assert_close(rowsum.cpu(), dy.to(dtype).float().sum(dim=(0, 2)).t(), 1e-4, "gconv rowsum")
    dW, dA = K.gconv_finish(dweff, Ad, Wd, sup, Cout, Cin)
    assert_close(dW, W.grad, tol, "gconv dW")
    # dA is produced on the graph's support (what A * edge_importance needs); off it, it is zero
    m = sup.mask.cpu().unsqueeze(0).expand_as(A)
    assert_close(dA.cpu()[m], A.grad[m], tol, "gconv dA")
    assert float(dA.cpu()[~m].abs().max()) == 0.0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Cin,Cout", [(64, 64), (128, 256), (24, 40)])
def test_gconv_weights_bias_one_launch(K, pkg, dtype, Cin, Cout):
    """stgcn_gconv_weights_bias (effective weights + the bias pushed through A in one launch) writes exactly
    what stgcn_gconv_weights and stgcn_gcn_bias write separately (same summation orders: bit-equal)."""
    torch.manual_seed(5)
    A0 = torch.tensor(pkg.Graph(**pkg.PKU_MMD).A, dtype=torch.float32)
    A = (A0 * (torch.rand(A0.shape) + 0.5)).to(DEV)
    P, V = A.shape[0], A.shape[-1]
    sup = K.GraphSupport(A)
    W = torch.randn(P * Cout, Cin, device=DEV)
    b = torch.randn(P * Cout, device=DEV)
    w_ref = K.gconv_weights(A, W, sup, Cout, Cin, False, dtype)
    b_ref = K.gcn_bias(A, b, 1, Cout)
    w_one, b_one = K.gconv_weights(A, W, sup, Cout, Cin, False, dtype, bias=b)
    torch.cuda.synchronize()
    for a in range(V):  # slots past deg[a] are never written (nor read by gconv)
        d = int(sup.deg[a])
        assert torch.equal(w_one[a, :d], w_ref[a, :d]), a
    assert torch.equal(b_one, b_ref.view(V, Cout))


@pytest.mark.parametrize("Cin,Cout", [(64, 64), (64, 128), (256, 256)])
def test_gconv_finish_bias_merged(K, pkg, Cin, Cout):
    """stgcn_gconv_wgrad_finish_bias (dW, dA and the bias through A in two launches, outputs overwritten) is
    bit-equal to stgcn_gconv_wgrad_finish into zeros followed by stgcn_gcn_bias_bwd, and stgcn_gconv_wgrad's
    one-launch slab + row-sum reduction gives the per-joint row sums of dy."""
    torch.manual_seed(6)
    A0 = torch.tensor(pkg.Graph(**pkg.PKU_MMD).A, dtype=torch.float32)
    A = (A0 * (torch.rand(A0.shape) + 0.5)).to(DEV).contiguous()
    P, V = A.shape[0], A.shape[-1]
    sup = K.GraphSupport(A)
    N, T = 4, 40
    x = torch.randn(N, Cin, T, V)
    dy = torch.randn(N, Cout, T, V)
    W = torch.randn(P * Cout, Cin, device=DEV) / Cin ** 0.5
    b = torch.randn(P * Cout, device=DEV)
    assert K.gconv_wgrad_rowsum_ok(sup, Cin, Cout, torch.bfloat16)
    S = torch.empty((V, Cout), device=DEV)
    dweff = K.gconv_wgrad(cl(x, torch.bfloat16), cl(dy, torch.bfloat16), sup, Cin, Cout, rowsum=S)
    assert_close(S.cpu(), dy.to(torch.bfloat16).float().sum(dim=(0, 2)).t(), 1e-4, "row sums")
    dW_ref, dA_ref = K.gconv_finish(dweff, A, W, sup, Cout, Cin)
    db_ref = K.gcn_bias_bwd(A, b, S, dA_ref, Cout)
    dW, dA, db = K.gconv_finish_bias(dweff, A, W, sup, Cout, Cin, b, S)
    torch.cuda.synchronize()
    assert torch.equal(dW, dW_ref) and torch.equal(dA, dA_ref) and torch.equal(db, db_ref)


@pytest.mark.parametrize("Cin,Cout", [(64, 64), (256, 256), (128, 64)])
def test_gconv_dgrad_masked_residual(K, pkg, Cin, Cout):
    """The data gradient with the identity residual's masked gradient added in its epilogue (res = (dy, sign
    bits)) is bit-identical to writing dz = dy * mask first and accumulating (the route it replaces)."""
    torch.manual_seed(11)
    A = torch.tensor(pkg.Graph(**pkg.PKU_MMD).A, dtype=torch.float32, device=DEV)
    P, V = A.shape[0], A.shape[-1]
    N, T = 2, 23
    bf = torch.bfloat16
    sup = K.GraphSupport(A)
    W = torch.randn(P * Cout, Cin, device=DEV) / Cin ** 0.5
    wT = K.gconv_weights(A, W, sup, Cout, Cin, True, bf)
    dg = cl(torch.randn(N, Cout, T, V), bf)
    dy = cl(torch.randn(N, Cin, T, V), bf)
    y = cl(torch.randn(N, Cin, T, V), bf)
    M = N * T * V
    rows = y.permute(0, 2, 3, 1).reshape(M, Cin)
    w8 = (2 ** torch.arange(8, device=DEV)).to(torch.uint8)
    bits = ((rows > 0).to(torch.uint8).view(M, Cin // 8, 8) * w8).sum(-1).to(torch.uint8)
    dz = (dy.float() * (y.float() > 0)).to(bf).contiguous(memory_format=torch.channels_last)
    ref = K.gconv(dg, wT, sup, Cout, Cin, trans=True, out=dz.clone(memory_format=torch.channels_last), accumulate=True)
    out = K.gconv(dg, wT, sup, Cout, Cin, trans=True, res=(dy, bits))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("Cin,Cout,N,T", [(64, 64, 8, 40), (256, 256, 8, 75), (128, 256, 4, 60)])
def test_gconv_wgrad_phases(K, pkg, Cin, Cout, N, T):
    """stgcn_gconv_wgrad split into its accumulation kernel (phase 1) and its slab reduction (phase 2) — what
    bench.py's roofline brackets — writes exactly what the one-call form (phase 0) writes, for a slab plan (64 -> 64,
    128 -> 256) and the wide plan (256 -> 256: 128 x 128 groups, two row parts merged in-kernel by the last arriver
    in part-index order, so the arrival order does not change a bit)."""
    import ctypes
    torch.manual_seed(9)
    A0 = torch.tensor(pkg.Graph(**pkg.PKU_MMD).A, dtype=torch.float32)
    sup = K.GraphSupport(A0.to(DEV))
    V = A0.shape[-1]
    x = cl(torch.randn(N, Cin, T, V), torch.bfloat16)
    dy = cl(torch.randn(N, Cout, T, V), torch.bfloat16)
    S0 = torch.empty((V, Cout), device=DEV)
    d0 = K.gconv_wgrad(x, dy, sup, Cin, Cout, rowsum=S0)
    L = pkg._lib
    outs = []
    for rep in range(2):  # twice: the split plan's arrival counters are zeroed per launch
        S = torch.empty((V, Cout), device=DEV)
        dweff = torch.empty_like(d0)
        d = L.GconvWgradDesc()
        d.rowsum = S.data_ptr()
        d.x, d.dy, d.nbr, d.deg, d.dweff = x.data_ptr(), dy.data_ptr(), sup.nbr.data_ptr(), sup.deg.data_ptr(), \
            dweff.data_ptr()
        d.NT, d.V, d.J, d.Cin, d.Cout, d.x_ld, d.dy_ld = N * T, V, sup.J, Cin, Cout, Cin, Cout
        nbytes = L.lib().stgcn_gconv_wgrad_workspace(d, 1)
        work = torch.empty(max(nbytes, 4) // 4, dtype=torch.float32, device=DEV)
        d.work, d.work_bytes = work.data_ptr(), nbytes
        for ph in (1, 2):
            d.phase = ph
            L.check(L.lib().stgcn_gconv_wgrad(ctypes.byref(d), 1, L.stream()), "gconv_wgrad")
        outs.append((dweff, S))
    torch.cuda.synchronize()
    for dweff, S in outs:
        assert torch.equal(dweff, d0) and torch.equal(S, S0)

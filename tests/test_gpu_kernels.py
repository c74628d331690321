"""Kernel-level numerics on the MI355X: each HIP entry point vs a plain PyTorch fp32 reference of
the same op (fp32 path: 1e-4 relative; bf16 path: 2e-2 relative).  Calls go through the C-ABI."""
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


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("cin,cout,kt,stride,T", [(64, 64, 9, 1, 37), (32, 128, 9, 2, 30), (16, 24, 1, 1, 11),
                                                  (128, 256, 9, 1, 12), (8, 64, 1, 1, 5), (64, 52, 1, 1, 1),
                                                  (24, 48, 9, 2, 11), (768, 256, 1, 1, 9), (256, 768, 1, 1, 9),
                                                  (256, 256, 9, 1, 10), (4, 8, 9, 2, 9), (64, 128, 1, 2, 21),
                                                  (128, 128, 9, 2, 31), (128, 256, 1, 2, 8), (256, 256, 9, 2, 20),
                                                  (128, 256, 9, 2, 30), (256, 128, 9, 2, 151)])
def test_conv_rows_fwd_and_trans(K, dtype, tol, cin, cout, kt, stride, T):
    torch.manual_seed(0)
    N, V = 3, 25
    pad = (kt - 1) // 2
    x = torch.randn(N, cin, T, V)
    w = torch.randn(cout, cin, kt, 1) / (cin * kt) ** 0.5
    b = torch.randn(cout)
    ref = F.conv2d(x, w, b, stride=(stride, 1), padding=(pad, 0))
    T_out = ref.shape[2]
    wp, cp, kp = K.pack_weight(w.squeeze(-1).permute(2, 0, 1).to(DEV), dtype, stride=stride)
    y = K.conv_rows(cl(x, dtype), wp, cin, cout, cp, kp, T, T_out, Kt=kt, stride=stride, pad=pad,
                    bias=b.to(DEV))
    assert_close(y.float(), ref, tol, "conv fwd")
    # transposed (data gradient)
    dy = torch.randn(ref.shape)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, b, stride=(stride, 1), padding=(pad, 0)).backward(dy)
    wtp, cq, kq = K.pack_weight(w.squeeze(-1).permute(2, 1, 0).to(DEV), dtype, stride=stride, trans=True)
    dx = K.conv_rows(cl(dy, dtype), wtp, cout, cin, cq, kq, T_out, T, Kt=kt, stride=stride, pad=pad, trans=True)
    assert_close(dx.float(), xr.grad, tol, "conv trans")


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("cin,cout,kt,stride,T", [(64, 64, 9, 1, 37), (32, 128, 9, 2, 30), (16, 24, 1, 1, 11),
                                                  (128, 64, 9, 1, 12), (24, 48, 9, 2, 11), (64, 64, 1, 2, 21),
                                                  (192, 64, 1, 1, 40), (256, 256, 9, 1, 10), (128, 256, 9, 2, 30),
                                                  (128, 128, 1, 2, 9), (96, 40, 9, 1, 3)])
def test_conv_wgrad(K, dtype, tol, cin, cout, kt, stride, T):
    torch.manual_seed(1)
    N, V = 3, 25
    pad = (kt - 1) // 2
    x = torch.randn(N, cin, T, V)
    w = (torch.randn(cout, cin, kt, 1) / (cin * kt) ** 0.5).requires_grad_(True)
    y = F.conv2d(x, w, None, stride=(stride, 1), padding=(pad, 0))
    dy = torch.randn(y.shape)
    y.backward(dy)
    dw = K.conv_wgrad(cl(x, dtype), cl(dy, dtype), cin, cout, T, y.shape[2], Kt=kt, stride=stride, pad=pad)
    assert_close(dw.cpu().permute(1, 2, 0).unsqueeze(-1), w.grad, tol, "wgrad")


@pytest.mark.parametrize("pro", [1, 2])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("stride", [1, 2])
def test_conv_wgrad_prologue(K, pro, dtype, tol, stride):
    """dW with the BatchNorm+ReLU (pro 1) or LayerNorm+ReLU (pro 2) prologue applied to the input."""
    torch.manual_seed(5)
    N, C, Co, T, V = 4, 64, 128, 33, 25
    x = torch.randn(N, C, T, V) * 1.5 + 0.3
    if pro == 1:
        pa, pb = torch.rand(C) + 0.5, torch.randn(C)
        h = torch.relu(x * pa.view(1, -1, 1, 1) + pb.view(1, -1, 1, 1))
        kw = dict(pro_a=pa.to(DEV), pro_b=pb.to(DEV))
    else:
        mu, rs = torch.randn(N, T), torch.rand(N, T) + 0.5
        pa, pb = torch.rand(C, V) + 0.5, torch.randn(C, V)
        h = torch.relu((x - mu.view(N, 1, T, 1)) * rs.view(N, 1, T, 1) * pa.view(1, C, 1, V) + pb.view(1, C, 1, V))
        kw = dict(pro_a=pa.reshape(-1).to(DEV), pro_b=pb.reshape(-1).to(DEV),
                  pro_stats=torch.stack([mu, rs], -1).reshape(-1, 2).to(DEV).contiguous())
    w = (torch.randn(Co, C, 9, 1) / 24).requires_grad_(True)
    y = F.conv2d(h, w, None, stride=(stride, 1), padding=(4, 0))
    dy = torch.randn(y.shape)
    y.backward(dy)
    dw = K.conv_wgrad(cl(x, dtype), cl(dy, dtype), C, Co, T, y.shape[2], Kt=9, stride=stride, pad=4, pro=pro, **kw)
    assert_close(dw.cpu().permute(1, 2, 0).unsqueeze(-1), w.grad, tol, "wgrad+prologue")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_prologue_bn_relu_and_stats(K, dtype):
    torch.manual_seed(2)
    N, C, T, V = 2, 64, 20, 25
    x = torch.randn(N, C, T, V) * 2 + 1
    sc, sh = torch.rand(C) + 0.5, torch.randn(C)
    w = torch.randn(C, C, 9, 1) / 24
    b = torch.randn(C)
    h = torch.relu(x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
    ref = F.conv2d(h, w, b, padding=(4, 0))
    wp, cp, kp = K.pack_weight(w.squeeze(-1).permute(2, 0, 1).to(DEV), dtype)
    st = torch.zeros((K.row_blocks(N * T * V, C), cp, 4), device=DEV)
    y = K.conv_rows(cl(x, dtype), wp, C, C, cp, kp, T, T, Kt=9, pad=4, bias=b.to(DEV), pro=1, pro_a=sc.to(DEV),
                    pro_b=sh.to(DEV), stats=st)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert_close(y.float(), ref, tol, "conv+prologue")
    mr, _, _ = K.bn_finalize(st, st.shape[0], cp, C, None, None)
    yr = y.float().cpu()
    mean = yr.mean(dim=(0, 2, 3))
    var = yr.var(dim=(0, 2, 3), unbiased=False)
    # stats come from the fp32 accumulators (before the bf16 rounding of the stored output)
    stol = 1e-4 if dtype == torch.float32 else 2e-3
    assert_close(mr[:, 0].cpu(), mean, stol, "bn mean")
    assert_close(mr[:, 1].cpu(), 1 / torch.sqrt(var + 1e-5), stol, "bn rstd")


@pytest.mark.parametrize("C,N,T", [(16, 2, 7), (64, 2, 7), (256, 2, 7), (4, 2, 7), (24, 3, 11), (8, 2, 9), (64, 6, 131),
                                   (16, 5, 97)])
@pytest.mark.parametrize("per_sample", [False, True])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
def test_amix(K, per_sample, dtype, tol, C, N, T):
    """A-mix forward / transposed / dA (jmix.hip, gcn_amix.hip) vs einsum; the larger cases give every wave
    of the jmix grid dozens of items across sample boundaries (its counted DMA/store waits)."""
    torch.manual_seed(3)
    V, P = 25, 3
    x = torch.randn(N, C, T, V)
    A = torch.randn((N, P, V, V) if per_sample else (P, V, V))
    xa = torch.einsum("nctv,npvw->npctw", x, A) if per_sample else torch.einsum("nctv,pvw->npctw", x, A)
    got = K.amix_fwd(cl(x, dtype), A.to(DEV).contiguous())
    assert_close(got.float().cpu().reshape(N, P, C, T, V), xa, tol, "amix fwd")
    dw = torch.randn(N, P, C, T, V)
    dw_cl = cl(dw.reshape(N, P * C, T, V), dtype)
    dx = K.cl_empty(N, C, T, V, dtype, DEV)
    K.amix_trans(dw_cl, A.to(DEV).contiguous(), C, dx, accumulate=False)
    ref_dx = torch.einsum("npctw,npvw->nctv", dw, A) if per_sample else torch.einsum("npctw,pvw->nctv", dw, A)
    assert_close(dx.float().cpu(), ref_dx, tol, "amix trans")
    dA = K.amix_dA(cl(x, dtype), dw_cl, A.to(DEV).contiguous())
    ref_dA = torch.einsum("nctv,npctw->npvw", x, dw)
    if not per_sample:
        ref_dA = ref_dA.sum(0)
    assert_close(dA.cpu(), ref_dA, tol, "amix dA")


@pytest.mark.parametrize("N,C,T,V", [(2, 96, 7, 25), (3, 48, 41, 25), (1, 4, 5, 3)])
def test_cast_colsum(K, N, C, T, V):
    """stgcn_cast_colsum: the bf16 copy of fp32 rows and their fp32 column sums (attention projections' backward,
    aagcn.py:139-141 autograd), against torch; run twice, bit-identical sums (fixed order)."""
    torch.manual_seed(11)
    x = torch.randn(N, C, T, V) * 3 + 1
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    out, cs = K.cast_colsum(xd, N * T * V, C)
    _, cs2 = K.cast_colsum(xd, N * T * V, C)
    assert torch.equal(out.cpu(), x.to(torch.bfloat16))
    assert_close(cs.cpu(), x.sum(dim=(0, 2, 3)), 1e-5, "column sums")
    assert torch.equal(cs, cs2)


def test_bn_kernels(K):
    torch.manual_seed(4)
    M, C = 5000, 64
    u = torch.randn(1, C, M, 1) * 3 + 2
    part, nb, _ = K.bn_stats_partial(cl(u), M, C)
    g, b = torch.rand(C) + 0.5, torch.randn(C)
    mr, sc, sh = K.bn_finalize(part, nb, C, C, g.to(DEV), b.to(DEV))
    ur = u.clone().requires_grad_(True)
    y = torch.relu(F.batch_norm(ur, None, None, g, b, training=True))
    dy = torch.randn(y.shape)
    y.backward(dy)
    yg = K.bn_apply(cl(u), sc, sh, M, C, relu=True)
    assert_close(yg.cpu(), y, 1e-5, "bn apply")
    sums = K.bn_bwd_reduce(cl(dy), M, C, mask=1, mref=yg, x=cl(u), mean_rstd=mr)
    dx = K.cl_empty(1, C, M, 1, torch.float32, DEV)
    K.bn_bwd_apply(cl(dy), M, C, dx, mask=1, mref=yg, x=cl(u), mean_rstd=mr, gamma=g.to(DEV), sums=sums)
    assert_close(dx.cpu(), ur.grad, 1e-4, "bn bwd")


def _padded_rows(t, dtype=torch.float32):
    """(N,C,T,V) channels-last view whose rows have one element of padding: an odd row stride, so the LayerNorm
    kernels take their scalar (unvectorised) path."""
    N, C, T, V = t.shape
    buf = torch.zeros(N, T, V, C + 1, dtype=dtype, device=DEV)
    buf[..., :C] = t.permute(0, 2, 3, 1).to(DEV, dtype)
    return buf[..., :C].permute(0, 3, 1, 2)


@pytest.mark.parametrize("C,padded", [(16, False), (256, True)])
def test_ln_kernels(K, C, padded):
    """LayerNorm stats / apply / backward (ln.hip) vs torch; C = 256 on rows with an odd stride is the scalar path
    at 1600 elements per frame (8 per thread of a 1024-thread block)."""
    torch.manual_seed(5)
    N, T, V = 3, 9, 25
    mk = _padded_rows if padded else cl
    x = torch.randn(N, C, T, V) * 2 - 1
    w, b = torch.rand(C, 1, V) + 0.5, torch.randn(C, 1, V) * 0.1
    xr = x.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    mean = xr.mean(dim=(1, 3), keepdim=True)
    var = xr.var(dim=(1, 3), keepdim=True)
    y = torch.relu(wr * (xr - mean) / torch.sqrt(var + 1e-5) + br)
    dy = torch.randn(y.shape)
    y.backward(dy)
    st = K.ln_stats(mk(x), N * T, V, C)
    yg = K.ln_apply(mk(x), st, w.reshape(-1).to(DEV), b.reshape(-1).to(DEV), N * T * V, V, C, relu=True)
    assert_close(yg.cpu(), y, 1e-5, "ln fwd")
    dx = mk(torch.zeros(N, C, T, V))
    dgb = torch.zeros(2, C * V, device=DEV)
    K.ln_bwd(mk(dy), mk(x), st, w.reshape(-1).to(DEV), b.reshape(-1).to(DEV), N * T, V, C, dx, mask=2, dgb=dgb)
    assert_close(dx.cpu(), xr.grad, 1e-4, "ln dx")
    assert_close(dgb[0].cpu().view(C, 1, V), wr.grad, 1e-4, "ln dgamma")
    assert_close(dgb[1].cpu().view(C, 1, V), br.grad, 1e-4, "ln dbeta")


def test_box_sum(K):
    torch.manual_seed(6)
    N, C, T, V = 2, 8, 30, 25
    x = torch.randn(N, C, T, V)
    for Kt, S in ((9, 1), (9, 2)):
        ref = torch.zeros_like(x)
        for i in range(Kt // S):
            ref[:, :, i * S:] += x[:, :, :T - i * S]
        assert_close(K.box_sum(cl(x), Kt, S).cpu(), ref, 1e-6, "box sum")
        adj = torch.zeros_like(x)
        for i in range(Kt // S):
            adj[:, :, :T - i * S] += x[:, :, i * S:]
        assert_close(K.box_sum(cl(x), Kt, S, trans=True).cpu(), adj, 1e-6, "box sum adjoint")


def _bn_ref(x, w, b):
    mu = x.mean(dim=(0, 2, 3), keepdim=True)
    var = x.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
    return (x - mu) / torch.sqrt(var + 1e-5) * w.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("mode", ["conv_res", "identity", "none", "bn1"])
def test_bn_bwd_fused(K, dtype, tol, mode):
    """Fused BN backward vs autograd of relu(BN2(u) + res) (stgcn.py:160-193) / relu(BN1(g)) (:152-153)."""
    torch.manual_seed(9)
    N, C, T, V = 3, 64, 21, 25
    M = N * T * V
    rnd = lambda t: t.to(dtype).float()  # inputs as the kernels store them (masks then agree exactly)
    u = rnd(torch.randn(N, C, T, V) * 2 + 0.5).requires_grad_(True)
    r = rnd(torch.randn(N, C, T, V) - 0.3).requires_grad_(True)
    x = rnd(torch.randn(N, C, T, V)).requires_grad_(True)
    w2, b2, wr, brr = torch.rand(C) + 0.5, torch.randn(C), torch.rand(C) + 0.5, torch.randn(C)
    w2.requires_grad_(True)
    b2.requires_grad_(True)
    if mode == "bn1":
        y = torch.relu(_bn_ref(u, w2, b2))
    else:
        res = {"conv_res": _bn_ref(r, wr, brr), "identity": x, "none": 0}[mode]
        y = torch.relu(_bn_ref(u, w2, b2) + res)
    dy = torch.randn(y.shape)
    y.backward(dy)

    def stats(t):
        return torch.stack([t.mean(dim=(0, 2, 3)), 1 / torch.sqrt(t.var(dim=(0, 2, 3), unbiased=False) + 1e-5)],
                           -1).to(DEV).contiguous()

    ud, rd = cl(u.detach(), dtype), cl(r.detach(), dtype)
    # the mask reference as the kernels see it: the stored (rounded) forward output
    yd = cl(y.detach(), dtype)
    du = torch.empty_like(ud)
    kw = dict(x1=ud, mr1=stats(u.detach()), g1=w2.detach().to(DEV), out1=du, bias_sums=True)
    if mode == "bn1":
        mr = stats(u.detach())
        sc = (w2.detach().to(DEV) * mr[:, 1])
        sh = (b2.detach().to(DEV) - mr[:, 0] * sc)
        kw.update(mask=2, mref=ud, msc=sc.contiguous(), msh=sh.contiguous())
    else:
        kw.update(mask=1, mref=yd)
    out2 = None
    if mode == "conv_res":
        out2 = torch.empty_like(rd)
        kw.update(x2=rd, mr2=stats(r.detach()), g2=wr.to(DEV), out2=out2)
    elif mode == "identity":
        out2 = torch.empty_like(ud)
        kw.update(out2=out2)
    sums, osum = K.bn_bwd_fused(cl(dy, dtype), M, C, **kw)
    assert_close(du.float(), u.grad, tol, "du")
    assert_close(osum[0].cpu(), u.grad.sum(dim=(0, 2, 3)), tol, "sum du", u.grad.abs().sum(dim=(0, 2, 3)).max())
    # the BN parameter gradients: sum dz = d beta2, sum dz*xhat1 = d gamma2
    assert_close(sums[0].cpu(), b2.grad, tol, "dbeta", b2.grad.abs().max() + 1e-3)
    assert_close(sums[1].cpu(), w2.grad, tol, "dgamma", w2.grad.abs().max() + 1e-3)
    if mode == "conv_res":
        assert_close(out2.float(), r.grad, tol, "dr")
    if mode == "identity":
        assert_close(out2.float(), x.grad, tol, "dx")


@pytest.mark.parametrize("cin,cout,T,N", [(128, 128, 37, 3), (256, 256, 23, 2), (128, 256, 16, 3), (256, 128, 150, 2)])
def test_conv_wide_prologue_stats(K, cin, cout, T, N):
    """The >= 128-channel Kt=9 stride-1 convs (conv_wide.hip, bf16): BN1+ReLU prologue, bias, BN2 partial
    statistics, and the transposed conv (data gradient), against torch fp32."""
    torch.manual_seed(3)
    V = 25
    x = torch.randn(N, cin, T, V) * 1.5 + 0.5
    sc, sh = torch.rand(cin) + 0.5, torch.randn(cin)
    w = torch.randn(cout, cin, 9, 1) / (cin * 9) ** 0.5
    b = torch.randn(cout)
    h = torch.relu(x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
    ref = F.conv2d(h, w, b, padding=(4, 0))
    wp, cp, kp = K.pack_weight(w.squeeze(-1).permute(2, 0, 1).to(DEV), torch.bfloat16)
    st = torch.zeros((K.row_blocks(N * T * V, cout), cp, 4), device=DEV)
    y = K.conv_rows(cl(x, torch.bfloat16), wp, cin, cout, cp, kp, T, T, Kt=9, pad=4, bias=b.to(DEV), pro=1,
                    pro_a=sc.to(DEV), pro_b=sh.to(DEV), stats=st)
    assert_close(y.float(), ref, 2e-2, "wide conv+prologue")
    mr, _, _ = K.bn_finalize(st, st.shape[0], cp, cout, None, None)
    yr = y.float().cpu()
    assert_close(mr[:, 0].cpu(), yr.mean(dim=(0, 2, 3)), 2e-3, "bn mean")
    assert_close(mr[:, 1].cpu(), 1 / torch.sqrt(yr.var(dim=(0, 2, 3), unbiased=False) + 1e-5), 2e-3, "bn rstd")
    dy = torch.randn(ref.shape)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, None, padding=(4, 0)).backward(dy)
    wtp, cq, kq = K.pack_weight(w.squeeze(-1).permute(2, 1, 0).to(DEV), torch.bfloat16)
    dx = K.conv_rows(cl(dy, torch.bfloat16), wtp, cout, cin, cq, kq, T, T, Kt=9, pad=4, trans=True)
    assert_close(dx.float(), xr.grad, 2e-2, "wide conv trans")


@pytest.mark.parametrize("cin,cout,T,N,stride", [(128, 128, 37, 3, 1), (256, 256, 23, 2, 1), (64, 256, 16, 3, 1),
                                                 (256, 128, 150, 2, 1), (128, 128, 300, 2, 2), (256, 256, 41, 2, 2),
                                                 (64, 128, 30, 3, 2)])
def test_wgrad_wide_prologue(K, cin, cout, T, N, stride):
    """>= 128-output-channel Kt=9 weight gradient (wgrad_wide.hip, frame ring, bf16; stride 2 folded into
    5 taps over frame pairs) with the BN1+ReLU prologue, against torch fp32."""
    torch.manual_seed(7)
    V = 25
    x = torch.randn(N, cin, T, V) * 1.5 + 0.3
    pa, pb = torch.rand(cin) + 0.5, torch.randn(cin)
    h = torch.relu(x * pa.view(1, -1, 1, 1) + pb.view(1, -1, 1, 1))
    w = (torch.randn(cout, cin, 9, 1) / (9 * cin) ** 0.5).requires_grad_(True)
    y = F.conv2d(h, w, None, stride=(stride, 1), padding=(4, 0))
    dy = torch.randn(y.shape)
    y.backward(dy)
    dw = K.conv_wgrad(cl(x, torch.bfloat16), cl(dy, torch.bfloat16), cin, cout, T, y.shape[2], Kt=9, stride=stride,
                      pad=4, pro=1, pro_a=pa.to(DEV), pro_b=pb.to(DEV))
    assert_close(dw.cpu().permute(1, 2, 0).unsqueeze(-1), w.grad, 2e-2, "wide wgrad+prologue")


@pytest.mark.parametrize("cin,cout,T,N", [(128, 128, 300, 2), (256, 256, 150, 2), (128, 256, 33, 3)])
def test_conv_wide_stride2_prologue_stats(K, cin, cout, T, N):
    """Stride-2 Kt=9 conv folded into a 5-tap conv over frame pairs (conv_wide.hip fold 1/2): BN1+ReLU
    prologue, bias, BN2 partials, and the data gradient, against torch fp32."""
    torch.manual_seed(4)
    V = 25
    x = torch.randn(N, cin, T, V) * 1.5 + 0.5
    sc, sh = torch.rand(cin) + 0.5, torch.randn(cin)
    w = torch.randn(cout, cin, 9, 1) / (cin * 9) ** 0.5
    b = torch.randn(cout)
    h = torch.relu(x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
    ref = F.conv2d(h, w, b, stride=(2, 1), padding=(4, 0))
    T_out = ref.shape[2]
    wp, cp, kp = K.pack_weight(w.squeeze(-1).permute(2, 0, 1).to(DEV), torch.bfloat16, stride=2)
    st = torch.zeros((K.row_blocks(N * T_out * V, cout), cp, 4), device=DEV)
    y = K.conv_rows(cl(x, torch.bfloat16), wp, cin, cout, cp, kp, T, T_out, Kt=9, stride=2, pad=4, bias=b.to(DEV),
                    pro=1, pro_a=sc.to(DEV), pro_b=sh.to(DEV), stats=st)
    assert_close(y.float(), ref, 2e-2, "s2 conv+prologue")
    mr, _, _ = K.bn_finalize(st, st.shape[0], cp, cout, None, None)
    yr = y.float().cpu()
    assert_close(mr[:, 0].cpu(), yr.mean(dim=(0, 2, 3)), 2e-3, "bn mean")
    assert_close(mr[:, 1].cpu(), 1 / torch.sqrt(yr.var(dim=(0, 2, 3), unbiased=False) + 1e-5), 2e-3, "bn rstd")
    dy = torch.randn(ref.shape)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, None, stride=(2, 1), padding=(4, 0)).backward(dy)
    wtp, cq, kq = K.pack_weight(w.squeeze(-1).permute(2, 1, 0).to(DEV), torch.bfloat16, stride=2, trans=True)
    dx = K.conv_rows(cl(dy, torch.bfloat16), wtp, cout, cin, cq, kq, T_out, T, Kt=9, stride=2, pad=4, trans=True)
    assert_close(dx.float(), xr.grad, 2e-2, "s2 conv trans")


@pytest.mark.parametrize("Cin,Nout", [(64, 96), (128, 192), (256, 384), (16, 8)])
def test_attn_proj(K, Cin, Nout):
    """stgcn_attn_proj: fp32 theta/phi from a bf16 activation with the weight split into two bf16 parts:
    within fp32 rounding of the fp32 product on the same (bf16-valued) inputs."""
    torch.manual_seed(Cin + Nout)
    N, T, V = 3, 37, 25
    x = torch.randn(N, Cin, T, V).to(torch.bfloat16)
    w = torch.randn(Nout, Cin) / Cin ** 0.5
    b = torch.randn(Nout) * 0.1
    ref = torch.einsum("oc,nctv->notv", w.double(), x.double()) + b.double().view(1, -1, 1, 1)
    got = K.attn_proj(cl(x.float(), torch.bfloat16), w.to(DEV), b.to(DEV))
    assert_close(got.cpu(), ref, 1e-5, "attn_proj")


@pytest.mark.parametrize("Cin,Cout,N,T", [(192, 64, 2, 64), (64, 96, 2, 64), (768, 256, 1, 64), (64, 64, 3, 37)])
def test_wgrad_1x1(K, Cin, Cout, N, T):
    """Kt = 1 weight gradient (wgrad1x1.hip split-K path when M % 32 == 0, the frame-tiled kernel otherwise):
    dW[co][ci] = sum over rows of dy[co] x[ci] on bf16 rows, fp32 accumulation; several chunks and groups."""
    torch.manual_seed(Cin + Cout + T)
    V = 25
    x = torch.randn(N, Cin, T, V).to(torch.bfloat16)
    dy = torch.randn(N, Cout, T, V).to(torch.bfloat16)
    ref = torch.einsum("nctv,notv->oc", x.double(), dy.double())
    dw = torch.zeros((1, Cout, Cin), device=DEV)
    got = K.conv_wgrad(cl(x.float(), torch.bfloat16), cl(dy.float(), torch.bfloat16), Cin, Cout, T, T, dw=dw)
    assert_close(got.reshape(Cout, Cin).cpu(), ref, 1e-4, "wgrad 1x1")


@pytest.mark.parametrize("mode", ["identity", "conv_res"])
def test_bn_apply_bits_and_mask3(K, mode):
    """bn_apply's sign-bit output (bit c % 8 of byte [m][c / 8] = stored y > 0) and the fused BN backward reading it
    as mask 3: bit-identical to mask 1 on the stored y (same dz, same sums, same outputs)."""
    torch.manual_seed(77)
    N, C, T, V = 3, 64, 23, 25
    M = N * T * V
    bf = torch.bfloat16
    u, x, r = (cl(torch.randn(N, C, T, V) * s + o, bf) for s, o in ((2, 0.3), (1, -0.2), (1, 0.1)))
    sc, sh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    rsc, rsh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    kw = dict(res_mode=2, r=r, rsc=rsc, rsh=rsh) if mode == "conv_res" else dict(res_mode=1, r=x)
    y_ref = K.bn_apply(u, sc, sh, M, C, **kw)
    bits = torch.empty((M, C // 8), dtype=torch.uint8, device=DEV)
    y = K.bn_apply(u, sc, sh, M, C, bits=bits, **kw)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    rows = y.permute(0, 2, 3, 1).reshape(M, C)
    expect = (rows > 0).to(torch.uint8).view(M, C // 8, 8)
    weights = (2 ** torch.arange(8, device=DEV)).to(torch.uint8)
    assert torch.equal(bits, (expect * weights).sum(-1).to(torch.uint8))
    dy = cl(torch.randn(N, C, T, V), bf)
    mr = torch.stack([torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5], 1).contiguous()
    gam = torch.rand(C, device=DEV) + 0.5
    outs = []
    for mk in (dict(mask=1, mref=y), dict(mask=3, mref=bits)):
        du, dx = torch.empty_like(u), torch.empty_like(u)
        extra = dict(x2=r, mr2=mr, g2=gam) if mode == "conv_res" else {}
        s, o = K.bn_bwd_fused(dy, M, C, x1=u, mr1=mr, g1=gam, out1=du, out2=dx, bias_sums=True, **extra, **mk)
        torch.cuda.synchronize()
        outs.append((du, dx, s.clone(), o.clone()))
    for a_, b_ in zip(outs[0], outs[1]):
        assert torch.equal(a_, b_)

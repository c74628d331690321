"""The frame-streaming 64-channel temporal conv (tconv_frame.hip) vs the row-conv kernels of the same op
(stgcn_conv_rows: conv_wide forward with the BN1 prologue, conv_persist data grad), and vs a plain PyTorch fp32
Conv2d((9, 1), padding (4, 0)) of relu(BN1(g)) (stgcn.py:151-159) on the same bf16 inputs."""
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


def cl(x, dtype=torch.bfloat16):
    return x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("N,T,V", [(2, 37, 25), (3, 8, 25), (64, 300, 25), (4, 21, 18), (65, 300, 25), (1, 1, 25)])
def test_tconv_frame_fwd_dgrad(K, N, T, V):
    torch.manual_seed(11)
    C = 64
    g = torch.randn(N, C, T, V).to(torch.bfloat16).float()
    W = torch.randn(C, C, 9, 1) * 0.05
    bt = torch.randn(C)
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.5
    h = torch.relu(g * sc.view(1, C, 1, 1) + sh.view(1, C, 1, 1)).to(torch.bfloat16).float()
    ref = F.conv2d(h, W, bt, padding=(4, 0))
    wt = W.squeeze(-1).to(DEV)
    wtp, cp, kp = K.pack_weight(wt.permute(2, 0, 1), torch.bfloat16, stride=1)
    st = torch.zeros((K.tconv_frame_row_blocks(N, T), cp, 4), device=DEV)
    u = K.tconv_frame(cl(g), wtp, cp, kp, bias=bt.to(DEV), pro_a=sc.to(DEV), pro_b=sh.to(DEV), stats=st)
    assert_close(u.float(), ref, 2e-2, "tconv_frame fwd")
    # the row-conv kernel of the same op (conv_wide at C = 64): the same rounding of h, so close to bf16 output
    st0 = torch.zeros((K.row_blocks(N * T * V, C), cp, 4), device=DEV)
    u0 = K.conv_rows(cl(g), wtp, C, C, cp, kp, T, T, Kt=9, stride=1, pad=4, bias=bt.to(DEV), stats=st0,
                     pro=1, pro_a=sc.to(DEV), pro_b=sh.to(DEV))
    assert_close(u.float(), u0.float(), 1e-2, "tconv_frame vs conv_rows fwd")
    mr, _, _ = K.bn_finalize(st, st.shape[0], cp, C, None, None)
    assert_close(mr[:, 0].cpu(), ref.mean(dim=(0, 2, 3)), 3e-3, "tconv_frame stats mean")
    assert_close(mr[:, 1].cpu(), 1.0 / (ref.var(dim=(0, 2, 3), unbiased=False) + 1e-5).sqrt(), 2e-2, "stats rstd")
    # data grad: dh = conv^T(du)
    du = torch.randn(N, C, T, V).to(torch.bfloat16).float()
    hr = h.clone().requires_grad_(True)
    F.conv2d(hr, W, None, padding=(4, 0)).backward(du)
    wtT, cq, kq = K.pack_weight(wt.permute(2, 1, 0), torch.bfloat16, stride=1, trans=True)
    dh = K.tconv_frame(cl(du), wtT, cq, kq, trans=True)
    assert_close(dh.float(), hr.grad, 2e-2, "tconv_frame dgrad")
    dh0 = K.conv_rows(cl(du), wtT, C, C, cq, kq, T, T, Kt=9, stride=1, pad=4, trans=True)
    assert_close(dh.float(), dh0.float(), 1e-2, "tconv_frame vs conv_rows dgrad")

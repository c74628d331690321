"""Temporal-conv weight gradient (stgcn_conv_wgrad, the tcn.2 weight path of stgcn.py:154-159) on the DMA-ring
kernel (wgrad_ring.hip: Kt = 9, stride 1, 64 / 128 output channels, bf16) vs autograd of F.conv2d in fp32 on the
same bf16-rounded operands: runs that do not divide T, a sample count that does not fill 256 blocks, the 18-joint
graph, both prologues (BatchNorm1 + ReLU recomputed from the pre-norm input, or none: LayerNorm's materialised h),
both output layouts (fresh nn.Conv2d order / accumulate into [Kt][Cout][Cin]), and bit-reproducibility.  N = 330 has
more than the ring kernel's 320 slab rows (one per sample at least): the call takes the bounded-workspace kernels."""
import pytest
import torch
import torch.nn.functional as F

from conftest import assert_close

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
BF = torch.bfloat16


@pytest.fixture(scope="module")
def K(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg.native


def cl(x, dtype=torch.float32):
    return x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)


def rb(t):
    return t.to(BF).float()


@pytest.mark.parametrize("Cin,Cout,N,T,V", [(64, 64, 3, 37, 25), (64, 64, 64, 300, 25), (128, 128, 5, 41, 18),
                                            (128, 128, 64, 150, 25), (128, 64, 2, 11, 25), (64, 128, 1, 70, 32),
                                            (64, 64, 330, 3, 25)])
@pytest.mark.parametrize("pro", [1, 0])
def test_wgrad_ring(K, Cin, Cout, N, T, V, pro):
    torch.manual_seed(300 + Cin + Cout + T + pro)
    x = rb(torch.randn(N, Cin, T, V) * 1.5 + 0.3)
    sc, sh = torch.rand(Cin) + 0.5, torch.randn(Cin) * 0.5
    h = rb(torch.relu(x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))) if pro else x
    dy = rb(torch.randn(N, Cout, T, V))
    w = torch.zeros(Cout, Cin, 9, 1, requires_grad=True)
    F.conv2d(h, w, None, padding=(4, 0)).backward(dy)
    kw = dict(Kt=9, stride=1, pad=4, pro=pro, pro_a=sc.to(DEV) if pro else None, pro_b=sh.to(DEV) if pro else None)
    dw = K.conv_wgrad_w(cl(x, BF), cl(dy, BF), Cin, Cout, T, T, **kw)
    assert_close(dw.cpu().unsqueeze(-1), w.grad, 1e-2, "wgrad ring (Conv2d order)")
    dw2 = K.conv_wgrad_w(cl(x, BF), cl(dy, BF), Cin, Cout, T, T, **kw)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2), "wgrad ring: not bit-reproducible"
    if N * T <= 400:  # out_mode 0: += into [Kt][Cout][Cin]
        base = torch.randn(9, Cout, Cin, device=DEV)
        acc = K.conv_wgrad(cl(x, BF), cl(dy, BF), Cin, Cout, T, T, dw=base.clone(), **kw)
        assert_close(acc.cpu(), base.cpu() + w.grad.squeeze(-1).permute(2, 0, 1), 1e-2, "wgrad ring (accumulate)")

"""Segmentation loss + statistics kernel (loss.hip) against the reference fixture (tests/golden/loss.npz,
generated from utils/loss.py) and the oracle (oracle.loss / oracle.statistics, loss.py:8-41,
statistics.py:5-16): all three output types, subsegment i > 0, the multi-block path at long trials, and
data-parallel shards whose losses sum to (and gradients equal) the single-process ones.
Tolerance: fp32, 1e-5 relative on the loss terms, 1e-5 of max|ref| on the gradients."""
import pytest
import torch

from conftest import assert_close, load_golden

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def P(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return pkg


@pytest.fixture(scope="module")
def LM(P):
    return P.loss


@pytest.fixture(scope="module")
def O():
    from oracle import stgcn_oracle
    return stgcn_oracle


def _ours(LM, i, logits, labels, class_dist, output_type="logits"):
    p = logits.to(DEV).requires_grad_(True)
    ce, mse = LM.Loss(DEV, class_dist, output_type)(i, p, labels.to(DEV))
    (ce + mse).backward()
    return ce.cpu(), mse.cpu(), p.grad.cpu()


def _ref(O, i, logits, labels, class_dist, output_type="logits"):
    p = logits.clone().double().requires_grad_(True)
    ce, mse = O.loss(i, p, labels, class_dist.double(), output_type)
    (ce + mse).backward()
    return ce.detach(), mse.detach(), p.grad


def test_loss_golden(LM):
    d = load_golden("loss")
    for i in (0, 1):
        labels = torch.from_numpy(d["labels%d" % i])
        ce, mse, g = _ours(LM, i, d["logits%d" % i], labels, d["class_dist"])
        assert_close(ce, d["ce%d" % i], 1e-5, f"ce{i}")
        assert_close(mse, d["mse%d" % i], 1e-5, f"mse{i}")
        assert_close(g, d["dlogits%d" % i], 1e-5, f"dlogits{i}")


@pytest.mark.parametrize("output_type", ["logits", "logsoftmax", "softmax"])
@pytest.mark.parametrize("i", [0, 1])
@pytest.mark.parametrize("L,C", [(64, 52), (7, 5), (300, 200), (6001, 52)])
def test_loss_vs_oracle(LM, O, output_type, i, L, C):
    g = torch.Generator().manual_seed(L * 7 + C)
    x = torch.randn(1, C, L, generator=g) * 3
    if output_type == "softmax":
        x = torch.softmax(x, dim=1)
    elif output_type == "logsoftmax":
        x = torch.log_softmax(x, dim=1)
    labels = torch.randint(0, C, (1, L - i), generator=g)
    cd = torch.rand(C, generator=g) * 100 + 1
    ce, mse, gr = _ours(LM, i, x, labels, cd, output_type)
    rce, rmse, rgr = _ref(O, i, x, labels, cd, output_type)
    assert_close(ce, rce, 1e-5, "ce")
    assert_close(mse, rmse, 1e-5, "mse")
    assert_close(gr, rgr, 1e-5, "dpred")


@pytest.mark.parametrize("i", [0, 1])
def test_statistics_vs_oracle(LM, O, i):
    g = torch.Generator().manual_seed(5)
    L, C = 500, 52
    x = torch.randn(1, C, L, generator=g)
    labels = torch.randint(0, C, (1, L - i), generator=g)
    labels[0, ::3] = torch.topk(x[:, :, i::3] if i == 0 else x[:, :, 1:][:, :, ::3], 5, dim=1)[1][0, 2]  # top-5 hits
    t1, t5, c1, c5, tot = LM.Statistics()(i, x.to(DEV), labels.to(DEV))
    r1, r5, rc1, rc5, rtot = O.statistics(i, x, labels)
    assert (c1, c5, tot) == (rc1, rc5, rtot)
    assert torch.equal(t1.cpu(), r1) and torch.equal(t5.cpu(), r5)


@pytest.mark.parametrize("world", [2, 3])
def test_loss_sharded_equals_whole(P, LM, O, world):
    """parallel.sharded_loss: each rank's (ce, mse) share sums to the whole trial's loss and the
    concatenated per-rank gradients are the single-process gradient (loss.py:25-41 over the full series)."""
    g = torch.Generator().manual_seed(11)
    L, C = 257, 52
    x = torch.randn(1, C, L, generator=g) * 2
    labels = torch.randint(0, C, (1, L), generator=g)
    cd = torch.rand(C, generator=g) * 100 + 1
    rce, rmse, rgr = _ref(O, 0, x, labels, cd)
    loss = LM.Loss(DEV, cd)
    parts_ce, parts_mse, grads = 0.0, 0.0, []
    for r in range(world):
        s, e = P.parallel.rank_slice(L, world, r)
        shard = P.parallel.SegmentShard.local(x.to(DEV), labels.to(DEV), loss.weight, s, e, L, r)
        p = x[:, :, s:e].to(DEV).requires_grad_(True)
        ce, mse = loss(0, p, labels[:, s:e].to(DEV), shard=shard)
        (ce + mse).backward()
        parts_ce += ce.item()
        parts_mse += mse.item()
        grads.append(p.grad.cpu())
    assert abs(parts_ce - rce.item()) <= 1e-5 * abs(rce.item())
    assert abs(parts_mse - rmse.item()) <= 1e-5 * abs(rmse.item())
    assert_close(torch.cat(grads, dim=2), rgr, 1e-5, "sharded dpred")

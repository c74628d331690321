"""The HIP model under data parallelism, on the GPU: two processes share the one MI355X of the test box
(gloo process group over HIP tensors — RCCL refuses two ranks on one device), each running the package's
HIP ``stgcn.Model`` (processor.py:32-33, 500-566).

* exchange path: every rank takes ``windows_for_rank`` of two unequal-length trials, computes its share of
  each trial's loss (``exchange_shard`` -> HIP ``loss.Loss`` via ``parallel.sharded_loss``) inside
  ``DistributedDataParallel`` with ``accumulate`` (no_sync on the first trial).  LayerNorm model: per-frame
  statistics, so the gradients must equal a single-process HIP run over the whole trials.  BatchNorm model:
  per-replica batch statistics (as the reference's DataParallel), so they must equal a single-process run
  that evaluates each rank's shard as its own batch.  fp32 and bf16.
* graph path: ``parallel.GraphedStep`` (the bench's --graph step: fwd + loss + bwd captured with the side
  stream as a parallel graph branch, flat all-reduce between the graphs) on each rank's own subsegment;
  the averaged gradient must equal the mean of the single-process per-subsegment gradients, and the graph
  replay must reproduce the eager step of the same rank.
"""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import ROOT, assert_grad_close, collect_ranks, reap_ranks

pytestmark = pytest.mark.gpu

W = 20
WORLD = 2


def _arch(norm):
    return {"strategy": "spatial", "in_feat": 3, "normalization": norm, "num_classes": 52, "output_type": "logits",
            "st-gcn": {"in_feat": 3, "layers": 2, "kernel": 9, "importance": True, "in_ch": [64, 64],
                       "out_ch": [64, 128], "stride": [1, 2], "residual": [1, 1], "dropout": [0, 0]}}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pkg():
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    return ge.load_package()


def _model(pkg, norm, dtype, dev):
    torch.manual_seed(5)
    m = pkg.MODELS["st-gcn"](rank=None, **dict(_arch(norm), graph=pkg.PKU_MMD))
    g = torch.Generator().manual_seed(6)
    with torch.no_grad():
        for p in m.edge_importance:
            p.add_(0.1 * torch.randn(p.shape, generator=g))
    return m.to(dev).set_compute_dtype(dtype)


def _trials():
    g = torch.Generator().manual_seed(9)
    return [(torch.randn(1, 3, L, 25, generator=g), torch.randint(0, 52, (1, L), generator=g)) for L in (13, 10)]


CLASS_DIST = torch.arange(1, 53, dtype=torch.float32)


def _grads(m):
    return {k: p.grad.detach().float().cpu().numpy() for k, p in m.named_parameters() if p.grad is not None}


def _exchange_worker(rank, world, port, q, norm, dtype):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        pkg = _pkg()
        par = pkg.parallel
        m = _model(pkg, norm, dtype, dev)
        dm = par.ddp(m, dev)
        crit = pkg.loss.Loss(dev, CLASS_DIST)
        trials = _trials()
        for k, (trial, labels) in enumerate(trials):
            L = trial.shape[2]
            s, e = par.rank_slice(L, world, rank)
            labels = labels.to(dev)
            with par.accumulate(dm, last=k == len(trials) - 1):
                x = par.windows_for_rank(trial.to(dev), W, world, rank)
                pred = dm(x).permute(2, 1, 0)                      # (1, 52, n): WindowSegment.mask_segment
                shard = par.exchange_shard(pred, labels, crit.weight, s, L)
                ce, mse = par.sharded_loss(crit, 0, pred, labels[:, s:e], shard, world)
                ((ce + mse) / len(trials)).backward()              # processor.py:538-541 (/ batch_size)
        torch.cuda.synchronize()
        q.put((rank, _grads(m)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _spawn(target, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, WORLD, port, q) + args) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    try:
        for r, g in collect_ranks(q, procs, WORLD, timeout=240):
            got[r] = g
    finally:
        reap_ranks(procs)
    for p in procs:
        assert p.exitcode == 0, f"rank process exited with {p.exitcode}"
    return got


def _single_exchange(pkg, norm, dtype, dev):
    """Single-process HIP reference of the exchange path: whole trials (LayerNorm) or each rank's shard as
    its own batch with the same loss shares (BatchNorm, per-replica statistics)."""
    par = pkg.parallel
    m = _model(pkg, norm, dtype, dev)
    crit = pkg.loss.Loss(dev, CLASS_DIST)
    trials = _trials()
    for trial, labels in trials:
        L = trial.shape[2]
        labels = labels.to(dev)
        if norm == "LayerNorm":
            x = par.windows_for_rank(trial.to(dev), W, 1, 0)
            ce, mse = crit(0, m(x).permute(2, 1, 0), labels)
            ((ce + mse) / len(trials)).backward()
            continue
        preds = []
        for r in range(WORLD):
            preds.append(m(par.windows_for_rank(trial.to(dev), W, WORLD, r)).permute(2, 1, 0))
        for r in range(WORLD):
            s, e = par.rank_slice(L, WORLD, r)
            prev = preds[r - 1][0, :, -1].detach() if r > 0 else None
            shard = par.SegmentShard(prev, crit.weight[labels.reshape(-1)].sum(), L - 1, r == 0)
            ce, mse = crit(0, preds[r], labels[:, s:e], shard=shard)
            ((ce + mse) / len(trials)).backward()  # = the DDP mean of the world-scaled shares
    torch.cuda.synchronize()
    return _grads(m)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("norm", ["LayerNorm", "BatchNorm"])
def test_ddp_hip_model_sharded_trials(pkg, norm, dtype):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    got = _spawn(_exchange_worker, norm, dtype)
    ref = _single_exchange(pkg, norm, dtype, torch.device("cuda", 0))
    tol = 1e-3 if dtype == "fp32" else 2e-2
    assert set(got[0]) == set(ref)
    for k in ref:
        # DDP all-reduced: both ranks hold the same gradient
        np.testing.assert_allclose(got[0][k], got[1][k], rtol=0, atol=1e-6 * max(1.0, np.abs(got[0][k]).max()))
        assert_grad_close(torch.from_numpy(got[0][k]), torch.from_numpy(ref[k]), tol, f"ddp {norm} {dtype} {k}",
                          reduction=True)


def _unit(rank):
    g = torch.Generator().manual_seed(40 + rank)
    return torch.randn(6, 3, W, 25, generator=g), torch.randint(0, 52, (1, 6), generator=g)


def _graph_worker(rank, world, port, q, bucketed=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        pkg = _pkg()
        m = _model(pkg, "BatchNorm", "bf16", dev)
        params = [p for p in m.parameters() if p.requires_grad]
        opt = torch.optim.SGD(params, lr=0.0)  # lr 0: the step leaves the parameters where the reference is
        crit = pkg.loss.Loss(dev, CLASS_DIST)
        x, labels = (t.to(dev) for t in _unit(rank))

        def fwd_loss():
            ce, mse = crit(0, m(x).permute(2, 1, 0), labels)
            return ce + mse

        opt.zero_grad(set_to_none=True)  # the rank's own (eager, local) gradient
        fwd_loss().backward()
        eager = _grads(m)
        if bucketed:  # the bucket mode's hooks and exchange, uncaptured (gloo cannot be captured)
            gstep = pkg.parallel.GraphedStep(fwd_loss, params, opt, world, bucket_mb=0.25, capture=False)
            assert len(gstep.buckets) > 1
        else:
            gstep = pkg.parallel.GraphedStep(fwd_loss, params, opt, world)
        for _ in range(2):
            gstep()
        torch.cuda.synchronize()
        q.put((rank, {"avg": _grads(m), "eager": eager}))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucketed", [False, True])
def test_graphed_step_flat_allreduce(pkg, bucketed):
    """GraphedStep at N = 2: captured fwd + loss + bwd, one flat all-reduce, captured optimizer — or (bucketed) the
    bucket mode's post-accumulate hooks issuing per-bucket all-reduces during the backward (run uncaptured: gloo);
    averaged gradient = mean of the per-rank gradients."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    got = _spawn(_graph_worker, bucketed)
    dev = torch.device("cuda", 0)
    refs = []
    for r in range(WORLD):
        m = _model(pkg, "BatchNorm", "bf16", dev)
        crit = pkg.loss.Loss(dev, CLASS_DIST)
        x, labels = (t.to(dev) for t in _unit(r))
        ce, mse = crit(0, m(x).permute(2, 1, 0), labels)
        (ce + mse).backward()
        refs.append(_grads(m))
    torch.cuda.synchronize()
    for k in refs[0]:
        mean = (refs[0][k] + refs[1][k]) / 2
        for r in range(WORLD):
            # eager step of the rank (same kernels, same process) vs the single-process run: identical inputs
            assert_grad_close(torch.from_numpy(got[r]["eager"][k]), torch.from_numpy(refs[r][k]), 1e-3,
                              f"eager rank {r} {k}", reduction=True)
            assert_grad_close(torch.from_numpy(got[r]["avg"][k]), torch.from_numpy(mean), 1e-3,
                              f"graph all-reduced {k}", reduction=True)


def _bucket_graph_worker(rank, world, port, q):
    """One rank, RCCL: GraphedStep's bucket mode (per-bucket all-reduces captured inside the one step graph, issued
    from the backward's post-accumulate hooks) against eager steps of the same model and optimizer."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        pkg = _pkg()
        res = {}
        x, labels = (t.to(dev) for t in _unit(0))
        for mode in ("eager", "graph"):
            m = _model(pkg, "BatchNorm", "bf16", dev)
            params = [p for p in m.parameters() if p.requires_grad]
            opt = pkg.optim.Adam(params, lr=1e-3)
            crit = pkg.loss.Loss(dev, CLASS_DIST)

            def fwd_loss():
                ce, mse = crit(0, m(x).permute(2, 1, 0), labels)
                return ce + mse

            losses = []
            if mode == "eager":
                for _ in range(4):
                    opt.zero_grad(set_to_none=False)
                    loss = fwd_loss()
                    loss.backward()
                    opt.step()
                    losses.append(float(loss))
            else:
                # 0.25 MB buckets: several buckets (and several captured collectives) for this small model
                gstep = pkg.parallel.GraphedStep(fwd_loss, params, opt, world, bucket_mb=0.25)
                res["n_buckets"] = len(gstep.buckets)
                losses.append(None)  # the constructor's eager step
                for _ in range(3):
                    losses.append(float(gstep()))
                gstep.remove_hooks()
            torch.cuda.synchronize()
            res[mode] = ({k: p.detach().float().cpu().numpy() for k, p in m.named_parameters()}, losses)
        q.put((rank, res))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_graphed_step_bucketed_allreduce_rccl(pkg):
    """GraphedStep(bucket_mb=...) on RCCL (one rank: the box has one GPU and RCCL refuses two ranks on it): the
    captured per-bucket collectives and the gradients as bucket views give the eager step's parameters and losses
    after 1 eager + 3 replayed steps."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_bucket_graph_worker, args=(0, 1, _free_port(), q))
    p.start()
    try:
        got = dict(collect_ranks(q, [p], 1, timeout=240))
    finally:
        reap_ranks([p])
    assert p.exitcode == 0
    res = got[0]
    assert res["n_buckets"] > 1
    pe, le = res["eager"]
    pg, lg = res["graph"]
    for a, b in zip(le[1:], lg[1:]):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (le, lg)
    for k in pe:
        np.testing.assert_allclose(pg[k], pe[k], rtol=1e-5, atol=1e-6, err_msg=k)

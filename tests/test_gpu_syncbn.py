"""Optional SyncBatchNorm (syncbn.py) on the GPU.

* ``stgcn_bn_merge``: the per-channel (count, mean, M2) entry it writes equals numpy's statistics of the rows,
  and finalizing a split list of merged entries gives what finalizing the whole partial list gives.
* model: two gloo ranks on the one MI355X of the test box (RCCL refuses two ranks on one device) each run
  the HIP ST-GCN (BatchNorm everywhere: input BatchNorm1d, norm1 / norm2, the residual conv's norm) under
  DistributedDataParallel with ``convert_sync_batchnorm``, on UNEQUAL shards of one batch.  Synchronised
  statistics make each rank's logits the matching rows of a single-process run over the whole batch, and
  the DDP-averaged gradient of the ranks' summed losses equal to that run's gradient / world size.  The same
  ranks without SyncBN (the reference's per-replica DataParallel semantics, the default) must NOT match
  (the test sees the statistics).  fp32 and bf16; plain batches, window-staged ones (WindowBatch, whose
  input norm statistics come from window.hip), the RT-ST-GCN training model (OfflineLayer's norms) and the
  AAGCN model (per-sample graphs through the A-first graph conv; fp32).
"""
import os

import numpy as np
import pytest
import torch

from conftest import assert_close, assert_grad_close, bn_fed_bias
from test_gpu_ddp import WORLD, _grads, _model, _pkg, _spawn

pytestmark = pytest.mark.gpu

N, T = 7, 20
SPLIT = (4, 3)   # unequal shards: the global count weights the ranks' statistics


def _batch():
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, 3, T, 25, generator=g)
    cap = torch.randn(1, 3, N + T - 1, 25, generator=g)   # window n = capture frames [n, n + T)
    return x, cap


def _rt_model(pkg, dtype, dev):
    from conftest import load_golden
    arch = dict(load_golden("rt_ref_strides")["arch"], normalization="BatchNorm")
    torch.manual_seed(5)
    m = pkg.MODELS["rt-st-gcn"](rank=None, **arch)
    return m.to(dev).set_compute_dtype(dtype)


def _aagcn_model(pkg, dtype, dev):
    arch = {"strategy": "spatial", "in_feat": 3, "output_type": "logits", "normalization": "BatchNorm",
            "num_classes": 52,
            "aa-gcn": {"layers": 2, "kernel": 9, "importance": True, "in_feat": 3, "in_ch": [64, 64],
                       "out_ch": [64, 128], "stride": [1, 2], "residual": [1, 1], "dropout": [0, 0]}}
    torch.manual_seed(5)
    m = pkg.MODELS["aa-gcn"](rank=None, **dict(arch, graph=pkg.PKU_MMD))
    return m.to(dev).set_compute_dtype(dtype)


def _make(pkg, route, dtype, dev):
    if route == "rt":
        return _rt_model(pkg, dtype, dev)
    if route == "aagcn":
        return _aagcn_model(pkg, dtype, dev)
    return _model(pkg, "BatchNorm", dtype, dev)


def _input(pkg, route, x, cap, s, e, dev):
    if route == "window":  # the window-staged norm_in + fcn_in (window.hip), statistics weighted per frame
        return pkg.segment.WindowBatch(cap.to(dev), s, e - s, T)
    return x[s:e].to(dev)


def _shard(rank):
    s = sum(SPLIT[:rank])
    return s, s + SPLIT[rank]


def _loss(out, s):
    """sum of the outputs against fixed weights that depend on the GLOBAL sample index (s = first sample)"""
    o = out.float().reshape(out.shape[0], -1)
    i = torch.arange(o.shape[1], device=o.device, dtype=torch.float32)
    n = torch.arange(s, s + o.shape[0], device=o.device, dtype=torch.float32)[:, None]
    return (o * torch.cos(0.37 * i + 1.3 * n)).sum()


def _sync_worker(rank, world, port, q, dtype, route):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        pkg = _pkg()
        x, cap = _batch()
        s, e = _shard(rank)
        xr = _input(pkg, route, x, cap, s, e, dev)
        res = {}
        # default: per-replica statistics
        m0 = _make(pkg, route, dtype, dev)
        with torch.no_grad():
            res["out_local"] = m0(xr).float().cpu().numpy()
        # SyncBN under DDP
        m = pkg.convert_sync_batchnorm(_make(pkg, route, dtype, dev))
        dm = pkg.parallel.ddp(m, dev)
        out = dm(xr)
        _loss(out, s).backward()
        torch.cuda.synchronize()
        res["out"] = out.detach().float().cpu().numpy()
        res["grads"] = _grads(m)
        q.put((rank, res))
        dist.barrier()
    finally:
        dist.destroy_process_group()


# AAGCN in fp32 only: its attention makes the model chaotic in its inputs (tests/test_aagcn_sensitivity.py), so two
# bf16 runs with different rounding orders are not comparable per rank
@pytest.mark.parametrize("dtype,route", [(d, r) for d in ("fp32", "bf16") for r in ("tensor", "window", "rt")]
                         + [("fp32", "aagcn")])
def test_syncbn_ddp_equals_single_process_batch(pkg, dtype, route):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    got = _spawn(_sync_worker, dtype, route)
    dev = torch.device("cuda", 0)
    x, cap = _batch()
    m = _make(pkg, route, dtype, dev)
    out = m(_input(pkg, route, x, cap, 0, N, dev))
    _loss(out, 0).backward()
    torch.cuda.synchronize()
    ref_out = out.detach().float().cpu()
    ref_g = _grads(m)
    tol = 1e-3 if dtype == "fp32" else 2e-2
    for r in range(WORLD):
        s, e = _shard(r)
        assert_close(torch.from_numpy(got[r]["out"]), ref_out[s:e], tol, f"syncbn {dtype} logits rank {r}")
        # per-replica statistics differ from the batch's: the comparison above is sensitive to the exchange
        scale = np.abs(ref_out.numpy()).max()
        d_sync = np.abs(got[r]["out"] - ref_out[s:e].numpy()).max() / scale
        d = np.abs(got[r]["out_local"] - ref_out[s:e].numpy()).max() / scale
        assert d > max(tol, 4 * d_sync), \
            f"rank {r}: per-replica logits as close to the global-statistics run ({d:.2e}) as SyncBN's ({d_sync:.2e})"
    assert set(got[0]["grads"]) == set(ref_g)
    for k in ref_g:
        g0, g1 = got[0]["grads"][k], got[1]["grads"][k]
        np.testing.assert_allclose(g0, g1, rtol=0, atol=1e-6 * max(1.0, np.abs(g0).max()))
        if bn_fed_bias(k):  # exact gradient 0 (a bias feeding batch statistics): rounding noise on both sides
            assert np.abs(g0 * WORLD).max() < 0.003 * np.abs(ref_g[k[:-4] + "weight"]).max(), k
            continue
        assert_grad_close(torch.from_numpy(g0) * WORLD, torch.from_numpy(ref_g[k]), tol, f"syncbn {dtype} {k}",
                          reduction=True)


def test_bn_merge_entries(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    K = pkg.native
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    C = 96
    rows = [torch.randn(M, C, generator=g) * 2.0 + torch.arange(C) * 0.1 for M in (5000, 1234)]
    merged, parts = [], []
    for xr in rows:
        xd = xr.to(dev).contiguous()
        part, nb, _ = K.bn_stats_partial(xd, xr.shape[0], C, ld=C)
        parts.append((part, nb))
        mg = K.bn_merge(part, nb, C, C)
        torch.cuda.synchronize()
        xn = xr.double().numpy()
        exp = np.stack([np.full(C, xr.shape[0]), xn.mean(0), ((xn - xn.mean(0)) ** 2).sum(0)], 1)
        np.testing.assert_allclose(mg[:, :3].cpu().double().numpy(), exp, rtol=2e-5, atol=1e-3)
        merged.append(mg)
    gam = torch.rand(C, generator=g).to(dev) + 0.5
    bet = torch.randn(C, generator=g).to(dev)
    # two "ranks": finalize over the gathered merged entries == finalize over the concatenated rows
    both = torch.stack(merged)                              # [2][C][4]
    mr, sc, sh = K.bn_finalize(both, 2, C, C, gam, bet)
    xa = torch.cat(rows).to(dev).contiguous()
    pa, nba, _ = K.bn_stats_partial(xa, xa.shape[0], C, ld=C)
    mr2, sc2, sh2 = K.bn_finalize(pa, nba, C, C, gam, bet)
    torch.cuda.synchronize()
    for a, b in ((mr, mr2), (sc, sc2), (sh, sh2)):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-5, atol=1e-5)

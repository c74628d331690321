"""Config 4 on the HIP path: the 9-layer config-2 model trained data-parallel on the
WindowSegment units of a long trial — the schedule ``bench.py --config 4`` times.

The reference trains a trial as subsegments of ``segment`` windows (processor.py:377-392, each a forward
with its own loss term ce/num_subsegments + mse/num_subsegments) and accumulates their gradients before the
optimizer step (processor.py:531-564).  ``parallel.segment_units`` lists the subsegments of every trial,
``units_for_rank`` deals them round-robin; each rank runs its units as ``segment.WindowBatch``es (64 or 65
windows of T = 300 frames staged on the GPU from the padded capture, window.hip) under
``parallel.accumulate`` (DDP.no_sync on all but the last micro-step).

Two processes share the test box's one GPU (gloo process group over HIP tensors; RCCL refuses two ranks on
one device).  Checked:
* every gradient after the all-reduce equals a single-process HIP accumulation over the same four units
  (DDP averages over the 2 ranks, so ×2) — fp32 at 1e-3, bf16 at 2e-2 (the same kernels on the same
  inputs; only the summation order of the all-reduce differs), and both ranks hold the same gradient;
* one unit's logits (the 65-window unit i = 1, with its overlap window) against the CPU oracle on the
  materialised windows, fp32 at 1e-3.
Trial lengths U[4000, 8000] with seed 2 (bench.trial_lengths); the first trial has ~94 units, so the four
units dealt first are units 0-3 of trial 0: i = 0 (64 windows) and i = 1, 2, 3 (65 windows each).
"""
import os
import random
import socket

import numpy as np
import pytest
import torch

from conftest import ROOT, assert_close, assert_grad_close, collect_ranks, reap_ranks

pytestmark = pytest.mark.gpu

WORLD = 2
T = 300
SEG = 64
UNITS_PER_RANK = 2
ARCH = {
    "strategy": "spatial", "in_feat": 3, "normalization": "BatchNorm", "num_classes": 52, "output_type": "logits",
    "st-gcn": {"in_feat": 3, "layers": 9, "kernel": 9, "importance": True,
               "in_ch": [64, 64, 64, 64, 128, 128, 128, 256, 256],
               "out_ch": [64, 64, 64, 128, 128, 128, 256, 256, 256],
               "stride": [1, 1, 1, 2, 1, 1, 2, 1, 1], "residual": [1] * 9, "dropout": [0] * 9},
}
CLASS_DIST = torch.arange(1, 53, dtype=torch.float32)


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


def _lengths():
    rng = random.Random(2)  # bench.trial_lengths: U[4000, 8000], seed 2
    return [rng.randint(4000, 8000) for _ in range(2)]


def _units(pkg, rank, world):
    units = pkg.parallel.segment_units(_lengths(), T, SEG)
    return pkg.parallel.units_for_rank(units, world, rank)[:UNITS_PER_RANK * (WORLD // world)]


def _trial(k, L):
    """Padded capture (1, 3, L + T - 1, 25) and labels (1, L) of trial k, identical in every process."""
    g = torch.Generator().manual_seed(700 + k)
    cap = torch.nn.functional.pad(torch.randn(1, 3, L, 25, generator=g), (0, 0, T - 1, 0))
    return cap, torch.randint(0, 52, (1, L), generator=g)


def _model(pkg, dtype, dev):
    torch.manual_seed(1538574472)
    m = pkg.MODELS["st-gcn"](rank=None, **dict(ARCH, graph=pkg.PKU_MMD))
    g = torch.Generator().manual_seed(6)
    with torch.no_grad():
        for p in m.edge_importance:
            p.add_(0.1 * torch.randn(p.shape, generator=g))
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    return m.to(dev).set_compute_dtype(dtype), sd


def _grads(m):
    return {k: p.grad.detach().float().cpu().numpy() for k, p in m.named_parameters() if p.grad is not None}


def _train_units(pkg, model, units, dev):
    """The bench's config-4 micro-steps over ``units`` (no optimizer step: the gradients are compared)."""
    crit = pkg.loss.Loss(dev, CLASS_DIST)
    lengths = _lengths()
    data = {}
    logits = {}
    for j, u in enumerate(units):
        if u.trial not in data:
            cap, lab = _trial(u.trial, lengths[u.trial])
            data[u.trial] = (cap.to(dev), lab.to(dev))
        cap, lab = data[u.trial]
        with pkg.parallel.accumulate(model, last=j == len(units) - 1):
            y = model(pkg.segment.WindowBatch(cap, u.n0, u.nw, T))
            ce, mse = crit(u.i, y.permute(2, 1, 0), lab[:, u.y0:u.y1])
            ((ce + mse) / u.count).backward()                    # processor.py:392 (/ num_subsegments)
        logits[u.i] = y.detach().float().cpu()
    torch.cuda.synchronize()
    return logits


def _worker(rank, world, port, q, dtype):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        pkg = _pkg()
        m, _ = _model(pkg, dtype, dev)
        dm = pkg.parallel.ddp(m, dev)
        units = _units(pkg, rank, world)
        assert len(units) == UNITS_PER_RANK
        _train_units(pkg, dm, units, dev)
        q.put((rank, [(u.trial, u.i, u.nw) for u in units], _grads(m)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _spawn(dtype):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q, dtype)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    try:
        for r, us, g in collect_ranks(q, procs, WORLD):
            got[r] = (us, g)
    finally:
        reap_ranks(procs)
    for p in procs:
        assert p.exitcode == 0, f"rank process exited with {p.exitcode}"
    return got


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_config4_units_ddp(pkg, dtype):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    got = _spawn(dtype)
    dev = torch.device("cuda", 0)
    # the units the ranks took, in deal order: 64-window first unit, then 65-window units with the overlap
    assert [u for r in range(WORLD) for u in got[r][0]] == [(0, 0, 64), (0, 2, 65), (0, 1, 65), (0, 3, 65)]
    m, sd = _model(pkg, dtype, dev)
    units = _units(pkg, 0, 1)
    assert [(u.trial, u.i) for u in units] == [(0, 0), (0, 1), (0, 2), (0, 3)]
    logits = _train_units(pkg, m, units, dev)
    ref = _grads(m)
    tol = 1e-3 if dtype == "fp32" else 2e-2
    assert set(got[0][1]) == set(ref)
    for k in ref:
        g0, g1 = got[0][1][k], got[1][1][k]
        np.testing.assert_allclose(g0, g1, rtol=0, atol=1e-6 * max(1.0, np.abs(g0).max()))
        # DDP averages over the ranks; the single process summed all four units
        assert_grad_close(torch.from_numpy(g0 * WORLD), torch.from_numpy(ref[k]), tol, f"config4 {dtype} {k}",
                          reduction=True)
    if dtype == "fp32":
        import sys
        sys.path.insert(0, ROOT)
        from oracle import stgcn_oracle as O
        u = units[1]
        cap, _ = _trial(u.trial, _lengths()[u.trial])
        x = pkg.segment.WindowBatch(cap, u.n0, u.nw, T).materialize()   # segment_generator.py:143
        with torch.no_grad():
            y_ref = O.stgcn_model(x, sd, dict(ARCH, graph=pkg.PKU_MMD))
        assert_close(logits[u.i], y_ref, 1e-3, "config4 unit i=1 logits vs oracle")

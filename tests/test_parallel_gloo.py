"""Multi-rank plumbing on the CPU (gloo, world_size 2): trial sharding covers every window / chunk
exactly once, the DDP wrapper's gradient all-reduce equals the single-process gradient of the union
batch, and the ST-GCN training step of a sharded trial — windows_for_rank -> model -> exchange_shard ->
per-rank loss share -> DDP all-reduce, with no_sync accumulation over two trials — reproduces the
single-process gradient of the reference loss over the whole trials (processor.py:531-564,
utils/loss.py:25-41).  The network here is the oracle's ST-GCN (LayerNorm config, per-frame statistics,
so sharding cannot change it) with the package Model's parameters: the HIP kernels need a GPU, and this
test is about the data-parallel path around them (parity of the kernels is the -m gpu suite's)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rank_slices_partition(pkg):
    par = pkg.parallel
    for n in (0, 1, 7, 300, 6001):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                s, e = par.rank_slice(n, world, r)
                got += list(range(s, e))
            assert got == list(range(n))


def test_windows_match_reference_unfold(pkg):
    par = pkg.parallel
    torch.manual_seed(0)
    L, W = 37, 10
    trial = torch.randn(1, 3, L, 25)
    # reference: F.pad(W-1 at the start) -> unfold(2, W, 1) -> permute -> (L, C, W, V) (segment_generator.py:143)
    ref = torch.nn.functional.pad(trial, (0, 0, W - 1, 0)).unfold(2, W, 1).permute(0, 2, 1, 4, 3)
    ref = ref.reshape(L, 3, W, 25)
    parts = [par.windows_for_rank(trial, W, 3, r) for r in range(3)]
    assert torch.equal(torch.cat(parts), ref)


def test_chunks_cover_with_overlap(pkg):
    par = pkg.parallel
    b = par.chunk_bounds(6000, 500, 8)
    assert b[0][0] == 0 and b[-1][1] == 6000
    for (s0, e0), (s1, e1) in zip(b, b[1:]):
        assert s1 == e0 - 8
    allc = sum((par.chunks_for_rank(6000, 500, 8, 4, r) for r in range(4)), [])
    assert allc == b


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    par = ge.load_package().parallel
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    m = par.ddp(model, torch.device("cpu"))
    x = torch.randn(8, 6, generator=torch.Generator().manual_seed(1))
    s, e = par.rank_slice(8, world, rank)
    loss = m(x[s:e]).pow(2).sum()
    loss.backward()
    if rank == 0:
        out.put([(p.grad * world).tolist() for p in model.parameters()])  # DDP averages
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_allreduce_matches_single_process(pkg):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    x = torch.randn(8, 6, generator=torch.Generator().manual_seed(1))
    model(x).pow(2).sum().backward()
    for g, p in zip(got, model.parameters()):
        assert torch.allclose(torch.tensor(g), p.grad, atol=1e-5)


LN_ARCH = {"strategy": "spatial", "in_feat": 3, "normalization": "LayerNorm", "num_classes": 52,
           "output_type": "logits",
           "st-gcn": {"in_feat": 3, "layers": 2, "kernel": 9, "importance": True, "in_ch": [8, 8],
                      "out_ch": [8, 16], "stride": [1, 2], "residual": [1, 1], "dropout": [0, 0]}}


class _OracleNet(torch.nn.Module):
    """The oracle ST-GCN as an nn.Module over the package Model's parameters (so DDP can wrap it)."""

    def __init__(self, pkg, O):
        super().__init__()
        torch.manual_seed(3)
        m = pkg.MODELS["st-gcn"](rank=None, **dict(LN_ARCH, graph=pkg.PKU_MMD))
        sd = m.state_dict()
        g = torch.Generator().manual_seed(4)
        for k, v in sd.items():
            if k.startswith("edge_importance"):
                sd[k] = v + 0.1 * torch.randn(v.shape, generator=g)
        self.names = list(sd)
        self.A = sd.pop("A")
        self.p = torch.nn.ParameterList([torch.nn.Parameter(sd[k].double()) for k in self.names if k != "A"])
        self.O = O
        self.arch = dict(LN_ARCH, graph=pkg.PKU_MMD)

    def forward(self, x):
        sd = dict(zip([k for k in self.names if k != "A"], self.p))
        sd["A"] = self.A.double()
        return self.O.stgcn_model(x, sd, self.arch)


def _trials():
    g = torch.Generator().manual_seed(9)
    out = []
    for L in (13, 10):  # unequal-length trials (README.md:139-145)
        out.append((torch.randn(1, 3, L, 25, generator=g, dtype=torch.float64), torch.randint(0, 52, (1, L), generator=g)))
    return out


W_WIN = 12
CLASS_DIST = torch.arange(1, 53, dtype=torch.float64)


def _model_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    from oracle import stgcn_oracle as O
    pkg = ge.load_package()
    par = pkg.parallel
    net = _OracleNet(pkg, O)
    m = par.ddp(net, torch.device("cpu"))
    w = 1 - CLASS_DIST / CLASS_DIST.sum()
    trials = _trials()
    for k, (trial, labels) in enumerate(trials):
        L = trial.shape[2]
        s, e = par.rank_slice(L, world, rank)
        with par.accumulate(m, last=k == len(trials) - 1):
            x = par.windows_for_rank(trial, W_WIN, world, rank)
            pred = m(x).permute(2, 1, 0)                       # (1, 52, n): WindowSegment.mask_segment
            shard = par.exchange_shard(pred, labels, w, s, L)
            ce, mse = O.loss_shard(0, pred, labels[:, s:e], CLASS_DIST, shard.prev, shard.den, shard.pairs,
                                   shard.rank_first)
            # DDP averages over ranks: scale the share by world; processor.py:538-541 divides by batch_size
            ((ce + mse) * world / len(trials)).backward()
    if rank == 0:
        out.put([p.grad.tolist() for p in net.p])
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_stgcn_step_matches_single_process(pkg):
    from oracle import stgcn_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_model_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    net = _OracleNet(pkg, O)
    trials = _trials()
    for trial, labels in trials:
        x = pkg.parallel.windows_for_rank(trial, W_WIN, 1, 0)
        ce, mse = O.loss(0, net(x).permute(2, 1, 0), labels, CLASS_DIST)
        ((ce + mse) / len(trials)).backward()
    for g, p in zip(got, net.p):
        g = torch.tensor(g, dtype=torch.float64)
        assert torch.allclose(g, p.grad, rtol=1e-7, atol=1e-10), (g - p.grad).abs().max()  # fp64 sum order


def test_segment_units_partition(pkg):
    """Config 4's units (parallel.segment_units) are exactly WindowSegment.get_segment's subsegments of each
    trial (segment_generator.py:132-145: window ranges, label ranges, index, count), and the round-robin deal
    gives every unit to exactly one rank with per-rank window counts within one unit of each other."""
    par, seg = pkg.parallel, pkg.segment
    lengths = [4123, 301, 7999, 64, 640]
    W, S = 300, 64
    units = par.segment_units(lengths, W, S)
    k = 0
    for t, L in enumerate(lengths):
        ws = seg.WindowSegment(staged=True, stages=1, num_classes=52, graph={"num_node": 25}, in_feat=3,
                               rank="cpu", world_size=1, receptive_field=W, segment=S)
        P0, _ = ws.pad_sequence(L)
        cap = torch.zeros(1, 3, L + P0, 25)
        lab = torch.zeros(1, L, dtype=torch.long)
        for i, (b, y, n) in enumerate(ws.get_segment(cap, lab)):
            u = units[k]
            assert (u.trial, u.i, u.count, u.n0, u.nw) == (t, i, n, b.n0, b.nw)
            assert u.y1 - u.y0 == y.shape[1] and u.nw == y.shape[1] + (1 if i > 0 else 0)
            k += 1
    assert k == len(units)
    for world in (1, 2, 3, 8):
        parts = [par.units_for_rank(units, world, r) for r in range(world)]
        assert sorted(id(u) for p in parts for u in p) == sorted(id(u) for u in units)
        assert max(len(p) for p in parts) - min(len(p) for p in parts) <= 1

"""Multi-rank plumbing on the CPU (gloo, world_size 2): trial sharding covers every window / chunk
exactly once, and the DDP wrapper's gradient all-reduce equals the single-process gradient of the
union batch (the data-parallel semantics the RCCL path uses on the GPU box)."""
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

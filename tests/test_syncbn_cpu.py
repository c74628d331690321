"""SyncBatchNorm plumbing on the CPU (syncbn.py): which modules ``convert_sync_batchnorm`` marks, that it leaves
the parameters and state_dict alone, and — over a gloo world of 2 — the backward-sum exchange: every rank ends
with the sums of all ranks scaled by M_rank / M_global (the apply kernels divide by their own M), in both the
count-lane form (the fused backward's float4 rows) and the packed form.  The statistics merge and the HIP
backward under real ranks are the -m gpu suite's (test_gpu_syncbn.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _arch(norm):
    return {"strategy": "spatial", "in_feat": 3, "normalization": norm, "num_classes": 52, "output_type": "logits",
            "st-gcn": {"in_feat": 3, "layers": 2, "kernel": 9, "importance": True, "in_ch": [64, 64],
                       "out_ch": [64, 128], "stride": [1, 2], "residual": [1, 1], "dropout": [0, 0]}}


def test_convert_marks_batchnorm_layers_only(pkg):
    m = pkg.MODELS["st-gcn"](rank=None, **dict(_arch("BatchNorm"), graph=pkg.PKU_MMD))
    keys = {k: v.clone() for k, v in m.state_dict().items()}
    pkg.convert_sync_batchnorm(m)
    marked = [n for n, mod in m.named_modules() if getattr(mod, "sync_bn", None) is not None]
    assert sorted(marked) == ["gcn_networks.0", "gcn_networks.1", "norm_in"], marked
    sd = m.state_dict()
    assert set(sd) == set(keys) and all(torch.equal(sd[k], keys[k]) for k in keys)
    # training only (torch.nn.SyncBatchNorm does not sync in eval)
    sync = pkg.syncbn.active_sync(m.gcn_networks[0])
    assert sync is not None
    m.eval()
    assert pkg.syncbn.active_sync(m.gcn_networks[0]) is None
    pkg.revert_sync_batchnorm(m.train())
    assert all(getattr(mod, "sync_bn", None) is None for mod in m.modules())
    ln = pkg.MODELS["st-gcn"](rank=None, **dict(_arch("LayerNorm"), graph=pkg.PKU_MMD))
    pkg.convert_sync_batchnorm(ln)
    assert not [n for n, mod in ln.named_modules() if getattr(mod, "sync_bn", None) is not None]


def test_world_requires_process_group(pkg):
    if dist.is_initialized():
        pytest.skip("a process group is already initialised")
    with pytest.raises(RuntimeError, match="not initialised"):
        pkg.syncbn.BnSync().world()


MS = (1000, 600)


def _rank_sums(rank, C=5):
    g = torch.Generator().manual_seed(10 + rank)
    return torch.randn(C, 4, generator=g), torch.randn(C, 2, generator=g)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from conftest import ROOT
        sys.path.insert(0, ROOT)
        import __graft_entry__ as ge
        pkg = ge.load_package()
        s4, s2 = _rank_sums(rank)
        sync = pkg.syncbn.BnSync()
        sync.all_reduce_sums(s4, MS[rank], count_lane=True)
        sync.all_reduce_sums(s2, MS[rank])
        q.put((rank, s4, s2))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_backward_sums_exchange_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        r, s4, s2 = q.get(timeout=120)
        got[r] = (s4, s2)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    tot4 = sum(_rank_sums(r)[0] for r in range(2))
    tot2 = sum(_rank_sums(r)[1] for r in range(2))
    Mg = float(sum(MS))
    for r in range(2):
        s4, s2 = got[r]
        torch.testing.assert_close(s4[:, :3], tot4[:, :3] * (MS[r] / Mg), rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(s4[:, 3], torch.full((5,), Mg))
        torch.testing.assert_close(s2, tot2 * (MS[r] / Mg), rtol=1e-6, atol=1e-6)

"""The 2-rank config-4 DDP run of tests/test_gpu_config4.py (gloo, both ranks on one GPU) with a check after every
unit's backward: prints any parameter gradient with non-finite or huge (> 1e6) entries, per rank and unit, and
whether it appeared before or after the all-reduce (the last unit).  Usage: python tools/debug_c4_ddp.py [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import test_gpu_config4 as C  # noqa: E402


def worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    msgs = []
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        pkg = C._pkg()
        m, _ = C._model(pkg, "bf16", dev)
        dm = pkg.parallel.ddp(m, dev)
        units = C._units(pkg, rank, world)
        crit = pkg.loss.Loss(dev, C.CLASS_DIST)
        lengths = C._lengths()
        cap, lab = C._trial(0, lengths[0])
        cap, lab = cap.to(dev), lab.to(dev)
        for j, u in enumerate(units):
            with pkg.parallel.accumulate(dm, last=j == len(units) - 1):
                y = dm(pkg.segment.WindowBatch(cap, u.n0, u.nw, C.T))
                ce, mse = crit(u.i, y.permute(2, 1, 0), lab[:, u.y0:u.y1])
                ((ce + mse) / u.count).backward()
            torch.cuda.synchronize()
            for k, p in m.named_parameters():
                if p.grad is None:
                    continue
                mx = p.grad.detach().abs().max().item()
                if not (mx < 1e6):
                    msgs.append(f"rank {rank} unit {j} (i={u.i}, nw={u.nw}) {k}: max|g| {mx:.3e}")
        q.put((rank, msgs))
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    ctx = mp.get_context("spawn")
    for rep in range(reps):
        q = ctx.Queue()
        port = C._free_port()
        procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
        for p in procs:
            p.start()
        out = [q.get(timeout=300) for _ in range(2)]
        for p in procs:
            p.join(timeout=60)
        bad = [m for _, ms in out for m in ms]
        print(f"rep {rep}: {len(bad)} bad", flush=True)
        for m in bad[:20]:
            print("  ", m, flush=True)

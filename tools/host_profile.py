"""Host-side cost of one config-2 training step (is the step host- or GPU-bound?): per phase host time
(forward enqueue, backward, optimizer) over K steps vs the wall time per step with the GPU in the loop.
Usage: python tools/host_profile.py [steps] [lean]   (lean: call torch._fused_adam_ on cached lists)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    pkg = ge.load_package()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = pkg.MODELS["st-gcn"](rank=None, **dict(bench.ARCH, graph=pkg.PKU_MMD)).to(dev).set_compute_dtype("bf16")
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.Adam(params, lr=5e-4, fused=True)
    x = torch.randn(bench.N_BATCH, 3, bench.T_LEN, bench.V_J, device=dev)
    labels = torch.randint(0, bench.CLASSES, (1, bench.N_BATCH), device=dev)
    crit = pkg.loss.Loss(dev, torch.rand(bench.CLASSES, device=dev) + 0.5)
    ph = {"zero": 0.0, "fwd": 0.0, "loss": 0.0, "bwd": 0.0, "opt": 0.0}

    def step(rec):
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        t1 = time.perf_counter()
        pred = model(x).permute(2, 1, 0)
        t2 = time.perf_counter()
        ce, mse = crit(0, pred, labels)
        loss = ce + mse
        t3 = time.perf_counter()
        loss.backward()
        t4 = time.perf_counter()
        opt.step()
        t5 = time.perf_counter()
        if rec:
            for k, a, b in (("zero", t0, t1), ("fwd", t1, t2), ("loss", t2, t3), ("bwd", t3, t4), ("opt", t4, t5)):
                ph[k] += b - a

    for _ in range(5):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    host = sum(ph.values()) / steps * 1e3
    print({k: round(v / steps * 1e3, 3) for k, v in ph.items()}, "host ms/step", round(host, 3), "wall ms/step",
          round(wall, 3), flush=True)
    if "cprofile" in sys.argv:  # where the host time goes (per-function own time over 10 steps)
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(10):
            step(False)
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(40)

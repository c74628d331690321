"""Where the step's small torch kernels come from: one config-2 step under torch.profiler, aten copy /
fill / mul / clone calls grouped by the innermost repository source line that issued them."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

if __name__ == "__main__":
    pkg = ge.load_package()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = pkg.MODELS["st-gcn"](rank=None, **dict(bench.ARCH, graph=pkg.PKU_MMD)).to(dev).set_compute_dtype("bf16")
    params = [p for p in model.parameters() if p.requires_grad]
    opt = pkg.optim.Adam(params, lr=5e-4)  # the bench step's optimizer
    x = torch.randn(bench.N_BATCH, 3, bench.T_LEN, bench.V_J, device=dev)
    labels = torch.randint(0, bench.CLASSES, (1, bench.N_BATCH), device=dev)
    crit = pkg.loss.Loss(dev, torch.rand(bench.CLASSES, device=dev) + 0.5)

    def step():
        opt.zero_grad(set_to_none=True)
        pred = model(x).permute(2, 1, 0)
        ce, mse = crit(0, pred, labels)
        (ce + mse).backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    want = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::mul", "aten::clone", "aten::add", "aten::sum",
            "aten::to", "aten::_to_copy", "aten::contiguous", "aten::zeros", "aten::mul_", "aten::add_", "aten::abs",
            "aten::eq", "aten::ne", "aten::div")
    cnt = collections.Counter()
    for ev in prof.events():
        if ev.name not in want:
            continue
        site = "?"
        for fr in ev.stack or []:
            if "realtime-st-gcn_amd" in fr or "tools/" in fr or "bench.py" in fr:
                site = fr.split("/root/repo/")[-1] if "/root/repo/" in fr else fr
                break
        cnt[(ev.name, site)] += 1
    for (name, site), n in cnt.most_common(60):
        print(f"{n:4d}  {name:18s} {site}")

"""Which repository lines issue the config-2 step's small torch kernels (copies, clones, fills, casts): one bench
step under a TorchDispatchMode that records the innermost repository frame of every such aten call on a HIP
tensor.   python tools/find_copies.py"""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

WANT = ("copy_", "clone", "_to_copy", "fill_", "zero_", "zeros", "ones", "full", "add_", "add", "mul", "mul_",
        "div_", "sum", "cat", "stack", "contiguous", "new_zeros", "empty_like")


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.cnt = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        if name in WANT:
            site = "?"
            for fr in reversed(traceback.extract_stack()):
                if "realtime-st-gcn_amd" in fr.filename or fr.filename.endswith("bench.py"):
                    site = f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.line.strip()[:70]}"
                    break
            self.cnt[(name, site)] += 1
        return func(*args, **(kwargs or {}))


if __name__ == "__main__":
    pkg = ge.load_package()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = pkg.MODELS["st-gcn"](rank=None, **dict(bench.ARCH, graph=pkg.PKU_MMD)).to(dev).set_compute_dtype("bf16")
    params = [p for p in model.parameters() if p.requires_grad]
    opt = pkg.optim.Adam(params, lr=5e-4)
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
    log = Log()
    with log:
        step()
    torch.cuda.synchronize()
    for (name, site), n in log.cnt.most_common(80):
        print(f"{n:4d}  {name:10s} {site}")

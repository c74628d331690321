"""Which Python line issues each device-side aten op (copies, fills, elementwise) in one config-2 training
step: a TorchDispatchMode logs every aten op on a CUDA tensor with the innermost package / bench frame.
    python tools/aten_trace.py"""
import os
import sys
import traceback
from collections import Counter

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

SKIP = {"aten.view.default", "aten.permute.default", "aten.select.int", "aten.slice.Tensor", "aten.empty.memory_format",
        "aten.empty_strided.default", "aten.as_strided.default", "aten.detach.default", "aten.unsqueeze.default",
        "aten.squeeze.dim", "aten.t.default", "aten._unsafe_view.default", "aten.unbind.int", "aten.expand.default",
        "aten.alias.default", "aten.empty_like.default", "aten.new_empty_strided.default", "aten.split.Tensor",
        "aten.split_with_sizes.default", "aten.transpose.int", "aten.squeeze.default", "aten.reshape.default",
        "aten.lift_fresh.default", "aten._to_copy.default_noop"}


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if name not in SKIP:
            fr = "?"
            for f in reversed(traceback.extract_stack()[:-1]):
                if "realtime-st-gcn_amd" in f.filename or "bench.py" in f.filename or "torch/optim" in f.filename:
                    fr = "%s:%d %s" % (os.path.basename(f.filename), f.lineno, f.line)
                    break
            if fr == "?":  # autograd-engine ops (no Python frame): identify by operand shapes / strides
                fr = " ".join("%s%s" % (tuple(t.shape), tuple(t.stride())) for t in args
                              if isinstance(t, torch.Tensor))[:110]
            self.c[(name, fr)] += 1
        return func(*args, **(kwargs or {}))


if __name__ == "__main__":
    P = ge.load_package()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = P.MODELS["st-gcn"](rank=None, **dict(bench.ARCH, graph=P.PKU_MMD)).to(dev).set_compute_dtype("bf16")
    params = [p for p in m.parameters() if p.requires_grad]
    opt = torch.optim.Adam(params, lr=5e-4, fused=True)
    x = torch.randn(64, 3, 300, 25, device=dev)
    labels = torch.randint(0, 52, (1, 64), device=dev)
    crit = P.loss.Loss(dev, torch.rand(52, device=dev) + 0.5)

    def step():
        opt.zero_grad(set_to_none=True)
        ce, mse = crit(0, m(x).permute(2, 1, 0), labels)
        (ce + mse).backward()
        opt.step()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    log = Log()
    with log:
        step()
    torch.cuda.synchronize()
    for (name, fr), n in log.c.most_common(60):
        print("%4d  %-36s %s" % (n, name, fr))

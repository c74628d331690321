"""Which Python lines launch the non-package (torch) kernels of the config-2 training step: torch.profiler over one
eager step of bench.py's model, the aten ops with a CUDA kernel grouped by their top package stack frames."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
import bench as B  # noqa: E402

pkg = ge.load_package()
dev = torch.device("cuda", 0)
torch.manual_seed(1538574472)
model = pkg.MODELS["st-gcn"](rank=None, **dict(B.ARCH, graph=pkg.PKU_MMD)).to(dev).set_compute_dtype("bf16")
params = [p for p in model.parameters() if p.requires_grad]
opt = pkg.optim.Adam(params, lr=5e-4)
crit = pkg.loss.Loss(dev, torch.rand(B.CLASSES, device=dev) + 0.5)
x = torch.randn(B.N_BATCH, 3, B.T_LEN, B.V_J, device=dev)
labels = torch.randint(0, B.CLASSES, (1, B.N_BATCH), device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    pred = model(x).permute(2, 1, 0)
    ce, mse = crit(0, pred, labels)
    (ce + mse).backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
for e in prof.key_averages(group_by_stack_n=6, group_by_input_shape=True):
    if not e.key.startswith("aten::") or e.device_time_total <= 0:
        continue
    if e.key in ("aten::empty", "aten::empty_strided"):
        continue
    st = [f for f in (e.stack or []) if "torch/" not in f][:4]
    print(f"{e.count:3d}x {e.key:24s} {e.device_time_total:8.1f}us {str(e.input_shapes)[:60]} | {' <- '.join(st)}")

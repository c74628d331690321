"""Which Python line launches each torch-side (non-stgcn) kernel of the config-2 training step: torch.profiler
over a few steps, aten ops that reach the device grouped by op and the first package/bench frame of their stack.
    python tools/torch_prof.py [steps]"""
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
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

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=25, max_name_column_width=30,
                                                      max_src_column_width=90))

"""Host-side cost of one config-2 training step (bench.py's eager step): CPU enqueue time vs GPU time,
and a cProfile of the Python launch path.   python tools/cpu_profile.py [steps]"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
pkg = ge.load_package()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = pkg.MODELS["st-gcn"](rank=None, **dict(bench.ARCH, graph=pkg.PKU_MMD)).to(dev).set_compute_dtype("bf16")
params = [p for p in model.parameters() if p.requires_grad]
opt = torch.optim.Adam(params, lr=5e-4, fused=True)
x = torch.randn(bench.N_BATCH, 3, bench.T_LEN, bench.V_J, device=dev)
labels = torch.randint(0, bench.CLASSES, (1, bench.N_BATCH), device=dev)
weight = torch.ones(bench.CLASSES, device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    loss = bench.loss_fn(model(x), labels, weight)
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
# enqueue-only time: the GPU queue is empty at the start, so this is the pure host cost of a step
enq = []
for _ in range(steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    enq.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
tot = (time.perf_counter() - t0) / steps
print(f"host enqueue per step: {1e3 * min(enq):.2f} ms (min) {1e3 * sum(enq) / len(enq):.2f} ms (mean); "
      f"pipelined step {1e3 * tot:.2f} ms")
pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)

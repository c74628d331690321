"""Time the one-launch weight preparation of the config-2 model (native.PrepPlan) and each of its jobs alone
(HIP events, 20 reps): which jobs bound the batched launch.  python tools/bench_prep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


if __name__ == "__main__":
    P = ge.load_package()
    K = P.native
    dev = torch.device("cuda", 0)
    m = P.MODELS["st-gcn"](rank=None, **dict(bench.ARCH, graph=P.PKU_MMD)).to(dev).set_compute_dtype("bf16")
    plan = m._prepared()
    print("whole plan: %d jobs, %d blocks, %.1f us" % (plan.njobs, plan.nblocks, timed(plan.run)))
    kinds = {0: "pack", 1: "s2frag", 2: "gconv", 3: "gbias"}
    for i, j in enumerate(plan._jobs):
        sub = K.PrepPlan(dev)
        sub._jobs = [j]
        sub._keep = plan._keep
        sub.finalize()
        print("job %2d %-6s trans %d Co %4d Ci %4d Kt %d threads %8d: %.1f us" %
              (i, kinds[j.kind], j.trans, j.Co, j.Ci, j.Kt, j.threads, timed(sub.run)))
    # every job of one kind (and direction) in one launch: which group bounds the batched launch
    groups = {}
    for j in plan._jobs:
        groups.setdefault((kinds[j.kind], j.trans), []).append(j)
    for (kn, tr), js in groups.items():
        sub = K.PrepPlan(dev)
        sub._jobs = js
        sub._keep = plan._keep
        sub.finalize()
        print("group %-6s trans %d: %2d jobs %5d blocks %.1f us" % (kn, tr, len(js), sub.nblocks, timed(sub.run)))

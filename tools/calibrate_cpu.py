"""CPU-baseline calibration: time the oracle (oracle/stgcn_oracle.py,
the CPU restatement bench.py runs on the GPU box as `cpu_baseline`, kind "port") against the REFERENCE
itself (imported from /root/reference — build container only, never on the GPU box) at identical shapes,
threads and weights, fwd + loss + bwd of the config-2 model (as_is st-gcn, 9 layers, BN, Kt=9).
Writes profiles/cpu_calibration.json: ratio = oracle time / reference time (same host).

    PYTHONDONTWRITEBYTECODE=1 python tools/calibrate_cpu.py [N] [reps]
"""
import copy
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, ROOT)
sys.path.insert(1, REF)

from models import MODELS  # noqa: E402  (reference, read-only)
from oracle import stgcn_oracle as O  # noqa: E402
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    threads = torch.get_num_threads()
    with open(os.path.join(REF, "config", "pku-mmd", "as_is", "stgcn_local.json")) as f:
        arch = json.load(f)["arch"]
    with open(os.path.join(REF, "data", "skeletons", "pku-mmd.json")) as f:
        arch["graph"] = json.load(f)
    arch["num_classes"] = bench.CLASSES
    torch.manual_seed(1538574472)
    ref = MODELS["st-gcn"](rank="cpu", **copy.deepcopy(arch))
    sd = {k: v.detach().clone().requires_grad_(v.dtype.is_floating_point) for k, v in ref.state_dict().items()}
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(n, 3, bench.T_LEN, bench.V_J, generator=gen)
    labels = torch.randint(0, bench.CLASSES, (1, n), generator=gen)
    weight = 1 - torch.rand(bench.CLASSES, generator=gen) / bench.CLASSES

    def t_ref():
        bench.loss_fn(ref(x), labels, weight).backward()

    def t_oracle():
        bench.loss_fn(O.stgcn_model(x, sd, arch), labels, weight).backward()

    out = {}
    for name, fn in (("reference", t_ref), ("oracle", t_oracle)):
        fn()  # warm-up
        best = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t0)
        out[name] = {"s_per_step": round(best, 4), "frames_per_s": round(n * bench.T_LEN / best, 1)}
    res = {"workload": f"config-2 model (as_is st-gcn, 9 layers, BN, Kt=9) fwd + loss + bwd, fp32, N={n} T=300 V=25",
           "host_cpu": bench.cpu_model(), "threads": threads, "torch": torch.__version__, **out,
           "ratio_oracle_over_reference": round(out["oracle"]["s_per_step"] / out["reference"]["s_per_step"], 4),
           "best_of": reps}
    print(json.dumps(res))
    with open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

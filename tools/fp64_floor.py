"""How far the reference's OWN fp32 gradients sit from the fp64 truth (the oracle run in float64 on the
golden inputs).  This is the accumulation-order floor any fp32 implementation shares: a HIP gradient
that needs the L2 criterion against the reference but whose error is of the same size as the
reference's own error is at that floor, not wrong.  Prints one line per tensor: max|ref32 - f64| /
max|f64| and the L2 relative error."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_golden, sub  # noqa: E402
from oracle import stgcn_oracle as O  # noqa: E402


def floor(case, run):
    d = load_golden(case)
    sd = {k: v.double().clone().requires_grad_(True) for k, v in sub(d, "sd/").items()}
    x = d["x"].double().clone().requires_grad_(True)
    y = run(x, sd, d)
    y.backward(d["dy"].double())
    rows = [("y", y.detach(), d["y"]), ("dx", x.grad, d["dx"])]
    rows += [(k, sd[k].grad, g) for k, g in sub(d, "grad/").items()]
    for name, truth, ref in rows:
        t = truth.double()
        r = ref.double()
        e = (r - t).abs().max().item() / max(t.abs().max().item(), 1e-30)
        l2 = ((r - t).norm() / max(t.norm().item(), 1e-30)).item()
        print(f"{case:32s} {name:36s} ref32-vs-f64 max/scale {e:.2e}  L2 {l2:.2e}")


if __name__ == "__main__":
    torch.set_num_threads(8)
    g = np.load(os.path.join(ROOT, "tests/golden/graphs.npz"))
    floor("model_aagcn_bn_narrow",
          lambda x, sd, d: O.aagcn_model(x, sd, d["arch"], torch.tensor(g["Araw/pku_mmd"][2]).double()))
    for c in ["stgcn_bn_1layer", "stgcn_bn_9layer_narrow", "stgcn_ln_9layer_narrow_k69"]:
        floor("model_" + c, lambda x, sd, d: O.stgcn_model(x, sd, d["arch"]))

"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE implementation.

Run ONLY in the build container (the reference is mounted read-only at
/root/reference and never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does: imports the reference's own nn.Modules (models/stgcn/stgcn.py,
models/rtstgcn/rtstgcn.py, models/aagcn/aagcn.py, models/utils/*.py,
utils/loss.py), runs them on seeded synthetic inputs on the CPU in fp32 and
stores inputs, parameters (under the reference's state_dict key names),
outputs and gradients as compressed .npz files.  Nothing from the reference
is copied: the fixtures are data only (inputs + expected outputs).

Reference bugs worked around here (documented in DESIGN.md):
  * OfflineLayer.forward multiplies by ``self.toeplitz`` which is never
    assigned (rtstgcn.py:368-379): we inject the Toeplitz matrix that the
    method builds locally (same recipe, rtstgcn.py:368-374) per layer.
  * OnlineLayer.eval_ (rtstgcn.py:522-525) is never called by the reference
    harness; we call it after _swap_layers_for_inference (rtstgcn.py:160-187)
    exactly as the docstring intends.
"""
import copy
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REF = os.environ.get("STGCN_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

from models import MODELS  # noqa: E402  (reference)
from models.stgcn.stgcn import StgcnLayer  # noqa: E402
from models.rtstgcn.rtstgcn import OfflineLayer  # noqa: E402
from models.aagcn.aagcn import AgcnLayer  # noqa: E402
from models.utils.graph import Graph  # noqa: E402
from models.utils.tgcn import ConvTemporalGraphical  # noqa: E402
from models.utils.layernorm import LayerNorm  # noqa: E402
from models.utils.batchnorm import BatchNorm1d  # noqa: E402
from utils.loss import Loss  # noqa: E402

torch.set_num_threads(8)


def skel(name):
    with open(os.path.join(REF, "data", "skeletons", name + ".json")) as f:
        return json.load(f)


def npf(t):
    return t.detach().cpu().numpy().astype(np.float32)


def perturb_norms(module, gen):
    """Give every norm affine a non-trivial value so affine paths are pinned."""
    with torch.no_grad():
        for name, p in module.named_parameters():
            if name.endswith("weight") and p.dim() in (1, 3) and ("norm" in name or "tcn.0" in name or "tcn.3" in name
                                                               or "residual.1" in name or "bn_relu" in name):
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=gen))
            elif name.endswith("bias") and p.dim() in (1, 3) and ("norm" in name or "tcn.0" in name or "tcn.3" in name
                                                                or "residual.1" in name or "bn_relu" in name):
                p.copy_(0.1 * torch.randn(p.shape, generator=gen))


def sd_np(module, prefix="sd/"):
    out = {}
    for k, v in module.state_dict().items():
        if torch.is_tensor(v):
            out[prefix + k] = npf(v)
    return out


def grads_np(module, prefix="grad/"):
    out = {}
    for k, p in module.named_parameters():
        if p.grad is not None:
            out[prefix + k] = npf(p.grad)
    return out


def save(name, d):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **d)
    print("wrote", path, "%.1f KB" % (os.path.getsize(path) / 1024))


# --------------------------------------------------------------------------- graphs
def make_graphs():
    d = {}
    for name in ["pku-mmd", "ntu-rgb+d", "openpose", "coco", "imu_fogit_ABCD", "hugadb"]:
        s = skel(name)
        g = Graph(strategy="spatial", **s)
        key = name.replace("+", "p").replace("-", "_")
        d["A/" + key] = g.A.astype(np.float64)
        d["Araw/" + key] = g.get_adjacency_raw().astype(np.float64)
        d["edge/" + key] = np.asarray(s["edge"], dtype=np.int64)
        d["meta/" + key] = np.asarray([s["num_node"], s["center"]], dtype=np.int64)
        for strat in ["distance", "uniform"]:
            d["A_%s/%s" % (strat, key)] = Graph(strategy=strat, **s).A.astype(np.float64)
    save("graphs", d)


# --------------------------------------------------------------------------- layers
def stgcn_layer_case(tag, cin, cout, stride, kt, norm, N=2, T=12, residual=True, seed=0):
    s = skel("pku-mmd")
    A = torch.tensor(Graph(strategy="spatial", **s).A, dtype=torch.float32)
    P, V = A.shape[0], A.shape[1]
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(seed + 100)
    layer = StgcnLayer(cin, cout, (kt, V), P, V, stride=stride, dropout=0, residual=residual,
                       normalization=norm)
    perturb_norms(layer, gen)
    M = 1.0 + 0.1 * torch.randn(P, V, V, generator=gen)
    x = torch.randn(N, cin, T, V, generator=gen).requires_grad_(True)
    Aeff = (A * M).requires_grad_(True)
    y = layer(x, Aeff)
    dy = torch.randn(y.shape, generator=gen)
    y.backward(dy)
    d = {"x": npf(x), "A": npf(A), "M": npf(M), "y": npf(y), "dy": npf(dy), "dx": npf(x.grad),
         "dAeff": npf(Aeff.grad),
         "cfg": np.asarray([cin, cout, stride, kt, 1 if norm == "LayerNorm" else 0, int(residual)], np.int64)}
    d.update(sd_np(layer))
    d.update(grads_np(layer))
    save("stgcn_layer_" + tag, d)


def tgcn_batched_case():
    s = skel("pku-mmd")
    A = torch.tensor(Graph(strategy="spatial", **s).A, dtype=torch.float32)
    P, V = A.shape[0], A.shape[1]
    torch.manual_seed(3)
    gen = torch.Generator().manual_seed(33)
    m = ConvTemporalGraphical(16, 24, V, P)
    x = torch.randn(2, 16, 10, V, generator=gen).requires_grad_(True)
    Ab = (A[None] + 0.05 * torch.randn(2, P, V, V, generator=gen)).requires_grad_(True)
    y = m(x, Ab)
    dy = torch.randn(y.shape, generator=gen)
    y.backward(dy)
    d = {"x": npf(x), "A": npf(Ab), "y": npf(y), "dy": npf(dy), "dx": npf(x.grad), "dA": npf(Ab.grad)}
    d.update(sd_np(m))
    d.update(grads_np(m))
    # shared (P,V,V) adjacency as well
    m.zero_grad()
    x2 = x.detach().clone().requires_grad_(True)
    A2 = A.clone().requires_grad_(True)
    y2 = m(x2, A2)
    y2.backward(dy)
    d.update({"y_shared": npf(y2), "dx_shared": npf(x2.grad), "dA_shared": npf(A2.grad),
              "A_shared": npf(A)})
    d.update(grads_np(m, "grad_shared/"))
    save("tgcn_batched", d)


def norms_case():
    torch.manual_seed(4)
    gen = torch.Generator().manual_seed(44)
    x = torch.randn(3, 8, 7, 25, generator=gen) * 2 + 0.5
    ln = LayerNorm([8, 1, 25])
    with torch.no_grad():
        ln.weight.copy_(1 + 0.1 * torch.randn(ln.weight.shape, generator=gen))
        ln.bias.copy_(0.1 * torch.randn(ln.bias.shape, generator=gen))
    xl = x.clone().requires_grad_(True)
    yl = ln(xl)
    dyl = torch.randn(yl.shape, generator=gen)
    yl.backward(dyl)
    bn = BatchNorm1d(3 * 25, track_running_stats=False)
    with torch.no_grad():
        bn.norm.weight.copy_(1 + 0.1 * torch.randn(75, generator=gen))
        bn.norm.bias.copy_(0.1 * torch.randn(75, generator=gen))
    xb = (torch.randn(4, 3, 11, 25, generator=gen) * 3 - 1).requires_grad_(True)
    yb = bn(xb)
    dyb = torch.randn(yb.shape, generator=gen)
    yb.backward(dyb)
    d = {"ln_x": npf(x), "ln_y": npf(yl), "ln_dy": npf(dyl), "ln_dx": npf(xl.grad),
         "bn_x": npf(xb), "bn_y": npf(yb), "bn_dy": npf(dyb), "bn_dx": npf(xb.grad)}
    d.update(sd_np(ln, "ln_sd/"))
    d.update(grads_np(ln, "ln_grad/"))
    d.update(sd_np(bn, "bn_sd/"))
    d.update(grads_np(bn, "bn_grad/"))
    save("norms", d)


# --------------------------------------------------------------------------- models
NARROW_IN = [8, 8, 8, 8, 16, 16, 16, 32, 32]
NARROW_OUT = [8, 8, 8, 16, 16, 16, 32, 32, 32]


def stgcn_arch(config, layers, narrow, kernel=None, widths=None):
    with open(os.path.join(REF, "config", "pku-mmd", config)) as f:
        arch = json.load(f)["arch"]
    arch = copy.deepcopy(arch)
    arch["graph"] = skel("pku-mmd")
    arch["num_classes"] = 52
    key = [k for k in ("st-gcn", "rt-st-gcn", "aa-gcn") if k in arch][0]
    conf = arch[key]
    if narrow:
        conf["in_ch"], conf["out_ch"] = list(NARROW_IN), list(NARROW_OUT)
    if widths is not None:
        conf["in_ch"], conf["out_ch"] = list(widths[0]), list(widths[1])
    if kernel is not None:
        conf["kernel"] = kernel
        if "kernel" in arch:
            arch["kernel"] = kernel
    if layers == 1:
        conf["layers"] = 1
        conf["in_ch"], conf["out_ch"] = [conf["in_ch"][0]], [conf["in_ch"][0]]
        conf["stride"], conf["residual"], conf["dropout"] = [1], [1], [0]
    return key, arch


def model_case(tag, config, layers, narrow, N=2, T=64, kernel=None, seed=1538574472, widths=None):
    key, arch = stgcn_arch(config, layers, narrow, kernel, widths)
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(7)
    m = MODELS[key](rank="cpu", **copy.deepcopy(arch))
    perturb_norms(m, gen)
    with torch.no_grad():
        if hasattr(m, "edge_importance") and isinstance(m.edge_importance, torch.nn.ParameterList):
            for p in m.edge_importance:
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=gen))
    x = torch.randn(N, 3, T, 25, generator=gen).requires_grad_(True)
    y = m(x)
    dy = torch.randn(y.shape, generator=gen)
    y.backward(dy)
    d = {"x": npf(x), "y": npf(y), "dy": npf(dy), "dx": npf(x.grad),
         "arch": np.frombuffer(json.dumps(arch).encode(), dtype=np.uint8)}
    d.update(sd_np(m))
    d.update(grads_np(m))
    save("model_" + tag, d)


def toeplitz(L, K, S):
    # recipe of rtstgcn.py:368-374 (the matrix the reference builds but never stores)
    t = torch.zeros(L, L)
    for i in range(K // S):
        t += F.pad(torch.eye(L - S * i), (i * S, 0, 0, i * S))
    return t


def rt_case(tag, strides, L=30, narrow=True, seed=11):
    key, arch = stgcn_arch("ln/rtstgcn_local.json", 9, narrow)
    arch[key]["stride"] = list(strides)
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(seed + 1)
    m = MODELS[key](rank="cpu", **copy.deepcopy(arch))
    perturb_norms(m, gen)
    with torch.no_grad():
        for layer in m.st_gcn:
            layer.edge_importance.copy_(1.0 + 0.1 * torch.randn(layer.edge_importance.shape, generator=gen))
    for layer in m.st_gcn:
        layer.toeplitz = toeplitz(L, layer.kernel_size, layer.stride)
    x = torch.randn(1, 3, L, 25, generator=gen).requires_grad_(True)
    y = m(x)
    dy = torch.randn(y.shape, generator=gen)
    y.backward(dy)
    d = {"x": npf(x), "y_offline": npf(y), "dy": npf(dy), "dx": npf(x.grad),
         "arch": np.frombuffer(json.dumps(arch).encode(), dtype=np.uint8)}
    d.update(sd_np(m))
    d.update(grads_np(m))
    # online, frame by frame (rtstgcn.py:160-187, 522-525, 528-627)
    m.eval()
    with torch.no_grad():
        m._swap_layers_for_inference()
        for layer in m.st_gcn:
            layer.eval_()
        outs = [m(x.detach()[:, :, i:i + 1]) for i in range(L)]
    d["y_online"] = npf(torch.cat(outs, dim=2))
    save("rt_" + tag, d)


def agcn_layer_case():
    s = skel("pku-mmd")
    A = torch.tensor(Graph(strategy="spatial", **s).A, dtype=torch.float32)
    P, V = A.shape[0], A.shape[1]
    torch.manual_seed(5)
    gen = torch.Generator().manual_seed(55)
    layer = AgcnLayer(16, 16, (9, V), P, 1, True, 0, V, normalization="BatchNorm")
    perturb_norms(layer, gen)
    with torch.no_grad():
        layer.B.copy_(0.05 * torch.randn(layer.B.shape, generator=gen))
    x = torch.randn(2, 16, 12, V, generator=gen).requires_grad_(True)
    y = layer(x, A)
    dy = torch.randn(y.shape, generator=gen)
    y.backward(dy)
    d = {"x": npf(x), "A": npf(A), "y": npf(y), "dy": npf(dy), "dx": npf(x.grad)}
    d.update(sd_np(layer))
    d.update(grads_np(layer))
    save("agcn_layer", d)


def loss_case():
    gen = torch.Generator().manual_seed(9)
    class_dist = torch.randint(1, 1000, (52,), generator=gen).float()
    loss = Loss("cpu", class_dist, "logits")
    d = {"class_dist": npf(class_dist)}
    for i in (0, 1):
        logits = torch.randn(1, 52, 40, generator=gen).requires_grad_(True)
        labels = torch.randint(0, 52, (1, 40 if i == 0 else 39), generator=gen)
        ce, mse = loss(i, logits, labels)
        (ce + mse).backward()
        d.update({"logits%d" % i: npf(logits), "labels%d" % i: labels.numpy(), "ce%d" % i: npf(ce),
                  "mse%d" % i: npf(mse), "dlogits%d" % i: npf(logits.grad)})
    save("loss", d)


def config1_cases():
    # BASELINE config 1 at its exact shape: 1-layer st-gcn, x (2, 3, 64, 25), as_is (BatchNorm) and ln (LayerNorm)
    model_case("stgcn_bn_1layer_t64", "as_is/stgcn_local.json", 1, False, T=64)
    model_case("stgcn_ln_1layer_t64", "ln/stgcn_local.json", 1, False, T=64)


if __name__ == "__main__":
    if sys.argv[1:] == ["config1"]:  # only the config-1 fixtures (the others are unchanged)
        config1_cases()
        sys.exit(0)
    config1_cases()
    make_graphs()
    norms_case()
    stgcn_layer_case("bn_s1", 16, 16, 1, 9, "BatchNorm")
    stgcn_layer_case("bn_s2", 16, 32, 2, 9, "BatchNorm", seed=1)
    stgcn_layer_case("ln_s1", 24, 24, 1, 9, "LayerNorm", seed=2)
    stgcn_layer_case("ln_s2", 24, 48, 2, 9, "LayerNorm", seed=3, T=11)
    stgcn_layer_case("bn_c64", 64, 64, 1, 9, "BatchNorm", seed=4, T=6)
    stgcn_layer_case("ln_k69", 8, 8, 1, 69, "LayerNorm", seed=5, T=80)
    # residual=False needs C_in == C_out in the reference (stgcn.py:184 mul_scalar keeps C_in)
    stgcn_layer_case("bn_nores", 16, 16, 1, 9, "BatchNorm", seed=6, residual=False)
    tgcn_batched_case()
    model_case("stgcn_bn_1layer", "as_is/stgcn_local.json", 1, False, T=32)
    model_case("stgcn_bn_9layer_narrow", "as_is/stgcn_local.json", 9, True)
    # oneDNN's conv backward hangs on this Kt=69 shape; the native aten path gives the same fp32 math
    with torch.backends.mkldnn.flags(enabled=False):
        model_case("stgcn_ln_9layer_narrow_k69", "ln/stgcn_local.json", 9, True, T=40,
                   widths=([4, 4, 4, 4, 8, 8, 8, 8, 8], [4, 4, 4, 8, 8, 8, 8, 8, 8]))
    model_case("aagcn_bn_narrow", "as_is/aagcn_local.json", 9, True, T=24)
    rt_case("stride1", [1] * 9)
    rt_case("ref_strides", [1, 1, 1, 2, 1, 1, 2, 1, 1])
    agcn_layer_case()
    loss_case()

"""Pin the CPU oracle (oracle/stgcn_oracle.py) to the reference-generated golden fixtures.

Every fixture was produced by the reference's own modules (tests/golden/make_golden.py);
if these pass, the oracle restates the reference on those inputs, forward AND backward.
"""
import numpy as np
import pytest
import torch

from conftest import assert_close, grad_floor, load_golden, sub
from oracle import stgcn_oracle as O

SKELS = ["pku_mmd", "ntu_rgbpd", "openpose", "coco", "imu_fogit_ABCD", "hugadb"]


@pytest.mark.parametrize("key", SKELS)
def test_graph_matches_reference(key):
    g = np.load("tests/golden/graphs.npz")
    V, center = g["meta/" + key]
    edge = g["edge/" + key].tolist()
    np.testing.assert_allclose(O.graph_A(V, edge, center), g["A/" + key], rtol=0, atol=1e-12)
    np.testing.assert_allclose(O.adjacency(V, edge, center), g["Araw/" + key], rtol=0, atol=0)
    for strat in ("distance", "uniform"):
        np.testing.assert_allclose(O.graph_A(V, edge, center, strategy=strat), g["A_%s/%s" % (strat, key)],
                                   rtol=0, atol=1e-12)


def test_pku_graph_known_values():
    """test_graph.py prints A for pku-mmd: shape (3,25,25), nnz [25,24,24], sum 369.148."""
    g = np.load("tests/golden/graphs.npz")
    A = O.graph_A(25, g["edge/pku_mmd"].tolist(), 20)
    assert A.shape == (3, 25, 25)
    assert [int((A[p] != 0).sum()) for p in range(3)] == [25, 24, 24]
    assert abs(A.sum() - 369.148) < 1e-3


def _grad_run(fn, inputs, dy):
    ins = [t.clone().requires_grad_(True) for t in inputs]
    y = fn(*ins)
    y.backward(dy)
    return y, [t.grad for t in ins]


def test_norms():
    d = load_golden("norms")
    ln = sub(d, "ln_sd/")
    y, (dx, dw, db) = _grad_run(lambda x, w, b: O.layernorm_cv(x, w, b), [d["ln_x"], ln["weight"], ln["bias"]],
                                d["ln_dy"])
    assert_close(y, d["ln_y"], 1e-5, "ln y")
    assert_close(dx, d["ln_dx"], 1e-5, "ln dx")
    assert_close(dw, d["ln_grad/weight"], 1e-5, "ln dw")
    bn = sub(d, "bn_sd/")
    y, (dx, dw, db) = _grad_run(lambda x, w, b: O.input_batchnorm(x, w, b),
                                [d["bn_x"], bn["norm.weight"], bn["norm.bias"]], d["bn_dy"])
    assert_close(y, d["bn_y"], 1e-5, "bn y")
    assert_close(dx, d["bn_dx"], 1e-5, "bn dx")
    assert_close(db, d["bn_grad/norm.bias"], 1e-5, "bn db")


LAYER_CASES = ["bn_s1", "bn_s2", "ln_s1", "ln_s2", "bn_c64", "ln_k69", "bn_nores"]


@pytest.mark.parametrize("case", LAYER_CASES)
def test_stgcn_layer(case):
    d = load_golden("stgcn_layer_" + case)
    cin, cout, stride, kt, is_ln, residual = [int(v) for v in d["cfg"]]
    kind = "LayerNorm" if is_ln else "BatchNorm"
    sd = {k: v.clone().requires_grad_(True) for k, v in sub(d, "sd/").items()}
    x = d["x"].clone().requires_grad_(True)
    Aeff = (d["A"] * d["M"]).requires_grad_(True)
    y = O.stgcn_layer(x, Aeff, sd, "", kt, stride, bool(residual), kind)
    assert_close(y, d["y"], 1e-5, "y")
    y.backward(d["dy"])
    assert_close(x.grad, d["dx"], 1e-4, "dx")
    assert_close(Aeff.grad, d["dAeff"], 1e-4, "dAeff")
    grads = sub(d, "grad/")
    for k, g in grads.items():
        assert_close(sd[k].grad, g, 1e-4, k, grad_floor(grads, k))


def test_tgcn_batched_and_shared():
    d = load_golden("tgcn_batched")
    for suffix, A, y, dx, dA, gp in (("", d["A"], d["y"], d["dx"], d["dA"], "grad/"),
                                     ("_shared", d["A_shared"], d["y_shared"], d["dx_shared"], d["dA_shared"],
                                      "grad_shared/")):
        w = d["sd/conv.weight"].clone().requires_grad_(True)
        b = d["sd/conv.bias"].clone().requires_grad_(True)
        x = d["x"].clone().requires_grad_(True)
        Ar = A.clone().requires_grad_(True)
        out = O.tgcn(x, w, b, Ar)
        assert_close(out, y, 1e-5, "y" + suffix)
        out.backward(d["dy"])
        assert_close(x.grad, dx, 1e-5, "dx" + suffix)
        assert_close(Ar.grad, dA, 1e-5, "dA" + suffix)
        assert_close(w.grad, d[gp + "conv.weight"], 1e-5, "dw" + suffix)
        assert_close(b.grad, d[gp + "conv.bias"], 1e-5, "db" + suffix)


@pytest.mark.parametrize("case", ["stgcn_bn_1layer", "stgcn_bn_1layer_t64", "stgcn_ln_1layer_t64", "stgcn_bn_9layer_narrow",
                                  "stgcn_ln_9layer_narrow_k69"])
def test_stgcn_model(case):
    d = load_golden("model_" + case)
    sd = {k: v.clone().requires_grad_(True) for k, v in sub(d, "sd/").items()}
    x = d["x"].clone().requires_grad_(True)
    y = O.stgcn_model(x, sd, d["arch"])
    assert_close(y, d["y"], 1e-4, "y")
    y.backward(d["dy"])
    assert_close(x.grad, d["dx"], 1e-3, "dx")
    grads = sub(d, "grad/")
    for k, g in grads.items():
        assert_close(sd[k].grad, g, 1e-3, k, grad_floor(grads, k))


@pytest.mark.parametrize("case", ["stride1", "ref_strides"])
def test_rt_offline_and_online(case):
    d = load_golden("rt_" + case)
    sd = {k: v.clone().requires_grad_(True) for k, v in sub(d, "sd/").items()}
    x = d["x"].clone().requires_grad_(True)
    y = O.rt_model_offline(x, sd, d["arch"])
    assert_close(y, d["y_offline"], 1e-4, "offline y")
    y.backward(d["dy"])
    assert_close(x.grad, d["dx"], 1e-3, "offline dx")
    grads = sub(d, "grad/")
    for k, g in grads.items():
        assert_close(sd[k].grad, g, 1e-3, k, grad_floor(grads, k))
    with torch.no_grad():
        yo = O.rt_model_online(d["x"], {k: v.detach() for k, v in sd.items()}, d["arch"])
    assert_close(yo, d["y_online"], 1e-4, "online y")


def test_agcn_layer():
    d = load_golden("agcn_layer")
    sd = {k: v.clone().requires_grad_(True) for k, v in sub(d, "sd/").items()}
    x = d["x"].clone().requires_grad_(True)
    y = O.agcn_layer(x, d["A"], sd, "", 9, 1, True, "BatchNorm", 3)
    assert_close(y, d["y"], 1e-5, "y")
    y.backward(d["dy"])
    assert_close(x.grad, d["dx"], 1e-4, "dx")
    grads = sub(d, "grad/")
    for k, g in grads.items():
        assert_close(sd[k].grad, g, 1e-4, k, grad_floor(grads, k))


def test_aagcn_model():
    d = load_golden("model_aagcn_bn_narrow")
    g = np.load("tests/golden/graphs.npz")
    sd = {k: v.clone().requires_grad_(True) for k, v in sub(d, "sd/").items()}
    x = d["x"].clone().requires_grad_(True)
    y = O.aagcn_model(x, sd, d["arch"], g["Araw/pku_mmd"][2])
    assert_close(y, d["y"], 1e-4, "y")
    y.backward(d["dy"])
    assert_close(x.grad, d["dx"], 1e-3, "dx")
    grads = sub(d, "grad/")
    for k, gr in grads.items():
        assert_close(sd[k].grad, gr, 1e-3, k, grad_floor(grads, k))


def test_loss():
    d = load_golden("loss")
    for i in (0, 1):
        logits = d["logits%d" % i].clone().requires_grad_(True)
        ce, mse = O.loss(i, logits, torch.from_numpy(d["labels%d" % i]), d["class_dist"])
        assert_close(ce, d["ce%d" % i], 1e-6, "ce")
        assert_close(mse, d["mse%d" % i], 1e-6, "mse")
        (ce + mse).backward()
        assert_close(logits.grad, d["dlogits%d" % i], 1e-5, "dlogits")

import json
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) and the built libstgcn_amd.so")


def load_golden(name):
    """Load a reference-generated fixture into torch tensors (safe loader: no pickle)."""
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    out = {}
    for k in d.files:
        v = d[k]
        if k == "arch":
            out[k] = json.loads(bytes(v.tolist()).decode())
        elif v.dtype == np.float32 or v.dtype == np.float64:
            out[k] = torch.from_numpy(v.copy())
        else:
            out[k] = v
    return out


def sub(d, prefix):
    return {k[len(prefix):]: v for k, v in d.items() if k.startswith(prefix)}


def _report(name, rel_max, tol, l2=None):
    """STGCN_TEST_REPORT=1: print every measured error (pytest -s) so tolerances stay evidence-based."""
    if os.environ.get("STGCN_TEST_REPORT"):
        extra = f" L2 {l2:.2e}" if l2 is not None else ""
        print(f"[err] {name}: max/scale {rel_max:.2e}{extra} (tol {tol:g})", flush=True)


def assert_close(got, ref, rel=1e-3, name="", scale_floor=0.0):
    """SURVEY §8(c) tolerance: max|got-ref| <= rel * max|ref| (plus a tiny absolute floor).

    ``scale_floor`` lifts the scale for tensors that are mathematically ~0 (e.g. the gradient of a
    conv bias that feeds a batch-statistics BatchNorm), whose reference values are rounding noise.
    """
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    assert got.shape == ref.shape, f"{name}: shape {tuple(got.shape)} != {tuple(ref.shape)}"
    scale = max(ref.abs().max().item(), scale_floor)
    err = (got - ref).abs().max().item()
    _report(name, err / max(scale, 1e-30), rel)
    assert err <= rel * scale + 1e-6, f"{name}: max err {err:.3e} > {rel:g} * {scale:.3e}"


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def pkg():
    import __graft_entry__ as ge
    return ge.load_package()


def grad_floor(grads, key):
    """Scale floor for a '.bias' grad: 1% of the paired '.weight' grad scale (see assert_close)."""
    if key.endswith("bias"):
        w = grads.get(key[:-4] + "weight")
        if w is not None:
            return 0.01 * w.abs().max().item()
    return 0.0


def bn_fed_bias(key):
    """Conv biases that feed a batch-statistics BatchNorm (tcn.2 -> tcn.3, residual.0 -> residual.1 of a BN
    StgcnLayer): their exact gradient is 0, so both the reference's and ours are rounding noise; they are
    checked against an absolute bound relative to the paired weight gradient instead of elementwise."""
    return key.endswith("tcn.2.bias") or key.endswith("residual.0.bias")


def assert_grad_close(got, ref, rel=1e-3, name="", scale_floor=0.0, reduction=False):
    """Gradient parity.  Max-norm ``rel`` as in assert_close, except that gradients downstream of a
    ReLU whose input is within rounding of 0 can legitimately flip (the reference's own CPU and GPU
    runs differ in the last bits; a flipped mask moves dy=O(1) into/out of the sum).  So: pass on the
    max-norm criterion, or on L2-relative <= 3*rel with at most 0.5% of elements beyond rel*max
    (``reduction=True``: weight / adjacency gradients sum over all rows, so a flip touches every
    element: L2 only)."""
    g = got.detach().double().cpu()
    r = ref.detach().double().cpu()
    assert g.shape == r.shape, f"{name}: shape {tuple(g.shape)} != {tuple(r.shape)}"
    scale = max(r.abs().max().item(), scale_floor)
    err = (g - r).abs()
    _report(name, err.max().item() / max(scale, 1e-30), rel,
            ((g - r).norm() / max(r.norm().item(), 1e-30)).item())
    if err.max().item() <= rel * scale + 1e-6:
        return
    l2 = ((g - r).norm() / max(r.norm().item(), 1e-30)).item()
    frac = (err > rel * scale + 1e-6).double().mean().item()
    if os.environ.get("STGCN_TEST_REPORT"):
        print(f"[l2-path] {name}: L2 {l2:.2e} frac beyond {frac:.2e} reduction={reduction}", flush=True)
    assert l2 <= 3 * rel and (frac <= 5e-3 or reduction), \
        f"{name}: max err {err.max().item():.3e} > {rel:g}*{scale:.3e}; L2 rel {l2:.2e}, frac beyond {frac:.2e}"


def collect_ranks(q, procs, n, timeout=300):
    """n results from the rank processes' queue; fails fast (instead of waiting out the timeout) when a rank
    process has died with an error."""
    import queue
    import time
    t0, out = time.time(), []
    while len(out) < n:
        try:
            out.append(q.get(timeout=5))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead:
                raise AssertionError(f"rank process exited with {dead[0]}")
            if time.time() - t0 > timeout:
                raise AssertionError("rank processes timed out")
    return out


def reap_ranks(procs):
    for p in procs:
        p.join(timeout=60)
    for p in procs:  # our own children only, by handle
        if p.is_alive():
            p.terminate()
            p.join(timeout=10)

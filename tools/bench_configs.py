"""SURVEY §8(d) configs 3 and 5 on one MI355X (synthetic data, random-init weights).

config 3: RT-ST-GCN online inference (config/pku-mmd/ln/rtstgcn_local.json: LN, K=9, 9 layers),
          one (1, 3, 1, 25) frame at a time through OnlineLayer FIFOs; per-frame latency p50/p99
          eager (one Python-launched kernel sequence per frame) and as a replayed HIP graph (the
          per-frame step captured once; FIFO state and indices are device buffers, so replays
          advance the stream correctly).  Parity of the two against each other is checked.
config 5: AAGCN (config/pku-mmd/as_is/aagcn_local.json: 2 streams, BN, 9 layers) fwd+bwd, bf16,
          N=64 T=300 V=25: skeleton-frames/s.
f1:       window staging (config/pku-mmd/ln/stgcn_local.json: receptive_field 50, segment 1000): norm_in +
          fcn_in of one segment's 1000 windows from the padded capture (window.hip) vs the reference's
          order (unfold the windows, then norm_in and fcn_in on the copies — our HIP kernels on both sides),
          fwd and bwd, BatchNorm and LayerNorm, bf16.

    python tools/bench_configs.py [--frames 2000] [--steps 10] [--only 3|5|ln|f1]
Prints one JSON line per config.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

LAYERS = {"layers": 9, "kernel": 9, "in_ch": [64, 64, 64, 64, 128, 128, 128, 256, 256],
          "out_ch": [64, 64, 64, 128, 128, 128, 256, 256, 256], "stride": [1, 1, 1, 2, 1, 1, 2, 1, 1],
          "residual": [1] * 9, "dropout": [0.0] * 9}
RT_ARCH = {"strategy": "spatial", "in_feat": 3, "stages": 1, "kernel": 9, "output_type": "logits",
           "normalization": "LayerNorm", "segment": 500, "num_classes": 52,
           "rt-st-gcn": dict(LAYERS, latency=False, importance=True, in_feat=3, buffer=1, stages=1)}
AAGCN_ARCH = {"strategy": "spatial", "receptive_field": 50, "in_feat": 3, "stages": 1, "output_type": "softmax",
              "normalization": "BatchNorm", "num_classes": 52,
              "aa-gcn": dict(LAYERS, latency=False, importance=True, in_feat=3, stages=1)}


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def config3(P, dev, frames):
    torch.manual_seed(0)
    m = P.MODELS["rt-st-gcn"](rank=None, **dict(RT_ARCH, graph=P.PKU_MMD)).to(dev)
    m.eval()
    m.prepare_benchmark(RT_ARCH)
    gen = torch.Generator(device=dev).manual_seed(3)
    stream = torch.randn(frames + 64, 1, 3, 1, 25, device=dev, generator=gen)
    R = P.routing.ROUTING
    prev = R.rt_one_launch
    try:
        R.rt_one_launch = False
        per_layer = _config3_route(m, stream, frames)
        R.rt_one_launch = True
        out = _config3_route(m, stream, frames)
    finally:
        R.rt_one_launch = prev
    out["per_layer_route"] = per_layer
    # workgroup count of the one-launch kernel: device time of 200 graph replays per count
    sweep = {}
    with torch.no_grad():
        for G in (16, 32, 64, 128, 256):
            m.reset_state()
            x_static = stream[0].clone()
            m(x_static)
            m._frame_pack[1][0].blocks = G
            g = torch.cuda.CUDAGraph()
            s_ = torch.cuda.Stream()
            s_.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s_):
                with torch.cuda.graph(g):
                    m(x_static)
            torch.cuda.current_stream().wait_stream(s_)
            for _ in range(20):
                g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            sweep[G] = round(e0.elapsed_time(e1) / 200, 4)
            assert int(m._frame_status.item()) == 0
        m._frame_pack[1][0].blocks = 0
    out["one_launch_blocks_device_ms"] = sweep
    return {"config": "3: rt-st-gcn online (ln/rtstgcn_local.json, LN, K=9, 9 layers), 1 frame (1,3,1,25)",
            "metric": "per-frame latency", "unit": "ms", "frames": frames, "dtype": "fp32",
            "route": "one persistent launch per frame (stgcn_rt_frame); per_layer_route: 2 launches per layer",
            "reference_cpu": "2.7 ms/frame (SURVEY §8(a12), 9 layers)", **out}


def _config3_route(m, stream, frames):
    out = {}
    with torch.no_grad():
        # eager: every kernel launched from Python per frame
        m.reset_state()
        lat, ys = [], []
        for i in range(frames):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            y = m(stream[i])
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0)
            if i < 64:
                ys.append(y.clone())
        warm = lat[32:]
        out["eager"] = {"p50_ms": round(1e3 * pct(warm, 0.5), 4), "p99_ms": round(1e3 * pct(warm, 0.99), 4)}
        # HIP graph: capture one per-frame step on a static input buffer, replay per frame
        m.reset_state()
        x_static = torch.zeros_like(stream[0])
        for i in range(3):  # warm-up launches (attribute setup, allocator) on the real stream
            x_static.copy_(stream[i])
            m(x_static)
        m.reset_state()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g):
                y_static = m(x_static)
        torch.cuda.current_stream().wait_stream(s)
        m.reset_state()  # the capture itself does not run the step
        lat, err = [], 0.0
        for i in range(frames):
            x_static.copy_(stream[i])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0)
            if i < 64:
                err = max(err, float((y_static - ys[i]).abs().max() / ys[i].abs().max().clamp_min(1e-12)))
        warm = lat[32:]
        out["graph"] = {"p50_ms": round(1e3 * pct(warm, 0.5), 4), "p99_ms": round(1e3 * pct(warm, 0.99), 4),
                        "max_rel_diff_vs_eager": err}
        # device time of one frame: HIP events around 200 back-to-back replays
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(200):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        out["graph"]["device_ms_per_frame"] = round(e0.elapsed_time(e1) / 200, 4)
    return out


def config5(P, dev, steps, warmup):
    torch.manual_seed(1538574472)
    m = P.MODELS["aa-gcn"](rank=None, **dict(AAGCN_ARCH, graph=P.PKU_MMD)).to(dev).set_compute_dtype("bf16")
    opt = P.optim.Adam(m.parameters(), lr=5e-4)  # the package's one-launch Adam (as bench.py)
    gen = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(64, 3, 300, 25, device=dev, generator=gen)
    labels = torch.randint(0, 52, (64,), device=dev, generator=gen)

    def step():
        y = m(x)
        loss = torch.nn.functional.nll_loss(torch.log(y.reshape(64, 52).clamp_min(1e-12)), labels)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"config": "5: aa-gcn (as_is/aagcn_local.json, 2 streams, BN, 9 layers) fwd+bwd+Adam, bf16, "
                      "N=64 T=300 V=25", "metric": "skeleton-frames/s", "value": round(steps * 64 * 300 / dt, 1),
            "ms_per_step": round(1e3 * dt / steps, 3), "steps": steps, "data": "synthetic"}


LN_ARCH = {"strategy": "spatial", "in_feat": 3, "normalization": "LayerNorm", "num_classes": 52,
           "output_type": "logits", "st-gcn": dict(LAYERS, importance=True, in_feat=3)}


def ln_train(P, dev, steps, warmup, reps=3, routes=(True, False)):
    """The LayerNorm st-gcn (ln/stgcn_vsc.json-style: LN, Kt = 9, config-2 widths) training step (fwd + loss +
    bwd + Adam, bf16, N=64 T=300) with its three 64 -> 64 layers' forward on the fused one-kernel layer
    (routing.fused_ln_train) and unfused (default), interleaved ``reps`` times."""
    R = P.routing.ROUTING
    torch.manual_seed(1538574472)
    m = P.MODELS["st-gcn"](rank=None, **dict(LN_ARCH, graph=P.PKU_MMD)).to(dev).set_compute_dtype("bf16")
    opt = P.optim.Adam(m.parameters(), lr=5e-4)
    gen = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(64, 3, 300, 25, device=dev, generator=gen)
    labels = torch.randint(0, 52, (1, 64), device=dev, generator=gen)
    crit = P.loss.Loss(dev, torch.rand(52, device=dev, generator=gen) + 0.5)

    def step():
        ce, mse = crit(0, m(x).permute(2, 1, 0), labels)
        (ce + mse).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    out = {"config": "ln st-gcn (LayerNorm, Kt=9, 9 layers, config-2 widths) fwd+loss+bwd+Adam, bf16, N=64 T=300",
           "metric": "ms/step"}
    prev = R.fused_ln_train
    try:
        for rep in range(reps):
            for route in routes:
                R.fused_ln_train = route
                for _ in range(warmup):
                    step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    step()
                torch.cuda.synchronize()
                k = "fused_ms_per_step" if route else "unfused_ms_per_step"
                out.setdefault(k, []).append(round(1e3 * (time.perf_counter() - t0) / steps, 3))
    finally:
        R.fused_ln_train = prev
    if "fused_ms_per_step" in out:
        out["fused_frames_per_s"] = round(64 * 300 / (min(out["fused_ms_per_step"]) * 1e-3), 1)
    return out


def staging(P, dev, reps=50):
    import torch.nn.functional as F
    W, nw, L, C, V, Cout = 50, 1000, 1000, 3, 25, 64
    gen = torch.Generator(device=dev).manual_seed(5)
    padded = F.pad(torch.randn(1, C, L, V, device=dev, generator=gen), (0, 0, W - 1, 0))
    w = torch.randn(Cout, C, 1, 1, device=dev, generator=gen).requires_grad_(True)
    b = torch.zeros(Cout, device=dev).requires_grad_(True)
    bf = torch.bfloat16
    out = {"config": "f1: window staging, 1000 windows x W=50 (ln/stgcn_local.json segment), C=3 -> 64, bf16",
           "out_bytes": nw * W * V * Cout * 2}
    for norm, mode in (("BatchNorm", 0), ("LayerNorm", 1)):
        if mode == 0:
            mod = P.BatchNorm1d(C * V).to(dev)
            gw, gb = mod.norm.weight, mod.norm.bias
        else:
            mod = P.LayerNorm([C, 1, V]).to(dev)
            gw, gb = mod.weight, mod.bias
        dy = torch.randn(nw, W, V, Cout, device=dev, generator=gen).to(bf).permute(0, 3, 1, 2)

        def staged():
            return P.layer_fn.WindowStageFunction.apply(padded, 0, nw, W, gw, gb, w, b, mode, bf)

        def unfolded():
            x = P.segment.WindowBatch(padded, 0, nw, W).materialize()
            x = mod(x)
            x = F.pad(x.permute(0, 2, 3, 1), (0, 8 - C)).permute(0, 3, 1, 2)
            return P.layer_fn.Conv1x1Function.apply(x, F.pad(w, (0, 0, 0, 0, 0, 8 - C)), b, bf)

        for name, fn in (("staged", staged), ("unfold_norm_conv", unfolded)):
            for _ in range(3):
                fn().backward(dy)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            tf = tb = 0.0
            for _ in range(reps):
                ev[0].record()
                y = fn()
                ev[1].record()
                y.backward(dy)
                ev[2].record()
                torch.cuda.synchronize()
                tf += ev[0].elapsed_time(ev[1])
                tb += ev[1].elapsed_time(ev[2])
            out["%s_%s_fwd_us" % (norm, name)] = round(1e3 * tf / reps, 1)
            out["%s_%s_bwd_us" % (norm, name)] = round(1e3 * tb / reps, 1)
        out["%s_staged_fwd_GBps" % norm] = round(out["out_bytes"] / (out["%s_staged_fwd_us" % norm] * 1e3), 1)
        out["%s_staged_bwd_GBps" % norm] = round(out["out_bytes"] / (out["%s_staged_bwd_us" % norm] * 1e3), 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--only", default=None)
    ap.add_argument("--ln-reps", type=int, default=3)
    ap.add_argument("--ln-route", choices=("both", "fused", "unfused"), default="both")
    args = ap.parse_args()
    P = ge.load_package()
    dev = torch.device("cuda", 0)
    if args.only in (None, "3"):
        print(json.dumps(config3(P, dev, args.frames)), flush=True)
    if args.only in (None, "5"):
        print(json.dumps(config5(P, dev, args.steps, args.warmup)), flush=True)
    if args.only in (None, "ln"):
        print(json.dumps(ln_train(P, dev, args.steps, args.warmup, args.ln_reps,
                                    {"both": (True, False), "fused": (True,), "unfused": (False,)}[args.ln_route])), flush=True)
    if args.only in (None, "f1"):
        print(json.dumps(staging(P, dev)), flush=True)


if __name__ == "__main__":
    main()

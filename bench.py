"""Benchmark: skeleton-frames/sec (fwd+bwd) of the 10-layer ST-GCN (fcn_in + 9 StgcnLayers, as_is BN,
Kt=9) at N=64 T=300 V=25 (BASELINE.json config 2), bf16 MFMA path, synthetic data.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--graph] [--config 2|4]

Config 2 (default): one step = forward of the whole model on one (64, 3, 300, 25) batch of windows + the
reference loss (weighted CE + clamped temporal MSE, utils/loss.py:25-41, windows as the time axis like
WindowSegment.mask_segment) + backward + Adam step.  Inputs are resident in HBM before timing.  Kernels are
launched eagerly from Python; --graph replays the step as HIP graphs (parallel.GraphedStep).
N > 1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) the ranks are the launcher's;
`python bench.py --gpus N` alone starts `torch.distributed.run --nproc-per-node N` as a child process
(before anything touches the GPU) and exits with its status.  Each rank trains on its own trial's
64-window subsegment (weak scaling; the subsegment's loss is self-contained, processor.py:377-392, so the
data path has no collective); gradients are averaged over ranks by DistributedDataParallel (RCCL
all-reduce in 4 MB buckets, ~4 for the 12.2 MB gradient, overlapped with backward) or, with --graph, by the same
4 MB bucket all-reduces captured inside the step's one HIP graph (parallel.GraphedStep bucket mode) — the
reference's accumulation of ``loss / batch_size`` over trials.

Config 4 (--config 4): the long-trial DDP workload of SURVEY 8(d): synthetic trials of U[4000, 8000]
frames (seed 2), cut into WindowSegment subsegments of 64 windows of T = 300 frames (the reference's
receptive-field windows at config 2's T), every subsegment a unit with its own loss term (ce + mse) /
num_subsegments; the units of all trials are dealt round-robin to the ranks
(parallel.segment_units / units_for_rank).  A step = one unit per rank (64-65 windows staged on the GPU
from the padded capture, window.hip), fwd + loss + bwd; the optimizer steps (and DDP all-reduces) every
--accum steps, DDP.no_sync on the others (processor.py:531-564).
Rank 0 prints ONE JSON line (metric/value/..., roofline, cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ARCH = {
    "strategy": "spatial", "in_feat": 3, "normalization": "BatchNorm", "num_classes": 52, "output_type": "logits",
    "st-gcn": {"in_feat": 3, "layers": 9, "kernel": 9, "importance": True,
               "in_ch": [64, 64, 64, 64, 128, 128, 128, 256, 256],
               "out_ch": [64, 64, 64, 128, 128, 128, 256, 256, 256],
               "stride": [1, 1, 1, 2, 1, 1, 2, 1, 1], "residual": [1] * 9, "dropout": [0] * 9},
}
N_BATCH, T_LEN, V_J, CLASSES = 64, 300, 25, 52
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 MFMA
HBM_PEAK_GBS = 8000.0


def loss_fn(logits, labels, weight):
    """utils/loss.py:25-41 with WindowSegment.mask_segment (N',C',1) -> (1,C',N') (segment_generator.py:151);
    CPU baseline only (the GPU step uses the HIP loss kernel, loss.Loss)."""
    pred = logits.permute(2, 1, 0)                      # (1, classes, windows)
    ce = torch.nn.functional.cross_entropy(pred, labels, weight=weight)
    ls = torch.log_softmax(pred, dim=1)
    mse = 0.15 * torch.clamp((ls[:, :, 1:] - ls.detach()[:, :, :-1]) ** 2, 0, 16).mean()
    return ce + mse


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def spawn_ranks(args):
    """`bench.py --gpus N` without a launcher: run torch.distributed.run as a child (this process has not
    touched the GPU) and return its exit status."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


# The roofline kernel (`roofline`): the step's largest kernel by time in the rocprofv3 summary,
# gconv_wgrad3_kernel — the graph-conv weight gradient dWeff[w][j] = dy[:, w]^T x[:, S(w)_j] (gconv.hip), 8
# launches per step (64->64 x3, 128->128 x2, 256->256 x2 as gconv_wgrad3w_kernel (128 x 128 groups), 128->256 x1; the
# 64->128 layer runs gconv_wgrad2).  Its C-ABI
# call is split (stgcn_gconv_wgrad_desc.phase) so HIP events bracket the kernel alone, not its slab reduction.
# Algorithmic work per launch: 2*N*T*nnz(S)*Cin*Cout flops over (x + dy) = N*T*V*(Cin+Cout)*2 bytes; the bound is the
# roof the launches' aggregate intensity falls under (HBM: ~228 flop/B < the ~312 ridge).
ROOF_KERNEL = "gconv_wgrad3"
ROOF_EVERY = 5  # timed steps per instrumented step (HIP events around the roofline launches)
# Secondary (`roofline_tcn_fwd`): conv_wide_kernel<128,9,8,1,0,64>, the Kt=9 stride-1 temporal-conv forward of the
# C=128 (T=150) and C=256 (T=75) layers, 4 launches per step.  Algorithmic work per launch = 2*N*T*V*C*C*Kt.
ROOF_TAGS = {"tcn_fwd_c128": 2.0 * N_BATCH * (T_LEN // 2) * V_J * 128 * 128 * 9,
             "tcn_fwd_c256": 2.0 * N_BATCH * (T_LEN // 4) * V_J * 256 * 256 * 9}


# north_star layer: StgcnLayer 64 -> 64, stride 1, Kt=9, BN, identity residual at N=64 T=300 V=25.
# Algorithmic forward work: 2NTV*Cin*P*Cout (gcn) + 2NP*Cout*T*V^2 (A-mix, dense as the
# reference counts it) + 2NTV*Cout^2*Kt (tcn) = 51.79 GFLOP.
LAYER_FWD_FLOP = (2.0 * N_BATCH * T_LEN * V_J * 64 * 3 * 64 + 2.0 * N_BATCH * 3 * 64 * T_LEN * V_J * V_J
                  + 2.0 * N_BATCH * T_LEN * V_J * 64 * 64 * 9)


def layer_roofline(pkg, dev, reps=20, norm="LayerNorm"):
    """Layer-level roofline of the north_star layer's forward (inference), timed with HIP events around every launch
    of the layer on the launch stream.  LayerNorm: the whole layer as the one fused kernel (layer_fused.hip) against
    the unfused forward of the same layer (routing.fused_inference off), plus the fused kernel's own launch time.
    BatchNorm: the unfused forward only — a BatchNorm layer has no one-kernel form (BN1's batch statistics need all
    of g first; the two-pass fused form lost to it and was removed in round 6), so ``fused_*`` is None."""
    K = pkg.native
    R = pkg.routing.ROUTING
    torch.manual_seed(0)
    A = torch.tensor(pkg.Graph(**pkg.PKU_MMD).A, dtype=torch.float32, device=dev)
    layer = pkg.StgcnLayer(64, 64, (9, V_J), A.shape[0], V_J, stride=1, normalization=norm).to(dev)
    pkg.set_compute_dtype(layer, "bf16")
    x = torch.randn(N_BATCH, 64, T_LEN, V_J, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ln = norm == "LayerNorm"
    kev = []

    def hook(tag, phase, work=None):
        if tag == "layer_fused":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.current_stream())
            kev.append(ev)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
        for _ in range(reps):
            fn()
        e1.record(torch.cuda.current_stream())
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    def graphed(fn):
        # the same forward captured once into a HIP graph and replayed: device time of the layer's kernels
        # without the per-launch host work of the eager Python path
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(st)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        return timed(g.replay)

    orig = K.layer_fused

    def tagged(*a, **k):
        k["tag"] = "layer_fused"
        return orig(*a, **k)

    prev_hook, prev_route = K.EVENT_HOOK, R.fused_inference
    fused_ms = fused_graph_ms = k_ms = None
    try:
        with torch.no_grad():
            if ln:
                K.layer_fused, K.EVENT_HOOK = tagged, hook
                R.fused_inference = True
                fused_ms = timed(lambda: layer(x, A))
                K.layer_fused, K.EVENT_HOOK = orig, prev_hook
                fused_graph_ms = graphed(lambda: layer(x, A))
            R.fused_inference = False
            unfused_ms = timed(lambda: layer(x, A))
            unfused_graph_ms = graphed(lambda: layer(x, A))
    finally:
        K.layer_fused, K.EVENT_HOOK, R.fused_inference = orig, prev_hook, prev_route
    pairs = [(kev[i], kev[i + 1]) for i in range(6, len(kev) - 1, 2)]  # skip the warm-up launches
    k_ms = sum(a.elapsed_time(b) for a, b in pairs) / len(pairs) if pairs else None

    def frac(ms):
        return None if ms is None else round(LAYER_FWD_FLOP / (ms * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS, 4)

    best = fused_ms if ln else unfused_ms
    achieved = LAYER_FWD_FLOP / (best * 1e-3) / 1e12
    return {"layer": f"StgcnLayer(64, 64, (9, 25), 3, 25, {norm}) forward, N=64 T=300 V=25, bf16 (north_star)",
            "path": "one fused kernel (layer_fused.hip)" if ln else "unfused (no one-kernel BatchNorm form)",
            "bound": "mfma", "algorithmic_gflop": round(LAYER_FWD_FLOP / 1e9, 2),
            "fused_fwd_ms": None if fused_ms is None else round(fused_ms, 4), "unfused_fwd_ms": round(unfused_ms, 4),
            "fused_kernel_ms": round(k_ms, 4) if k_ms else None,
            "achieved": round(achieved, 2), "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / BF16_DENSE_PEAK_TFLOPS, 4), "unfused_frac": frac(unfused_ms),
            "graph": {"fused_fwd_ms": None if fused_graph_ms is None else round(fused_graph_ms, 4),
                      "unfused_fwd_ms": round(unfused_graph_ms, 4), "frac": frac(fused_graph_ms if ln else unfused_graph_ms),
                      "unfused_frac": frac(unfused_graph_ms)}}


RIDGE_FLOP_PER_BYTE = BF16_DENSE_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)  # ~312 flop/B


def gwgrad_roofline(gw, world):
    """`roofline` of the dominant kernel (ROOF_KERNEL) from its live HIP-event pairs: (tag, ms, work) per launch,
    work = {"flop", "bytes", "shape"} (algorithmic).  Bound = the roof the aggregate intensity falls under; both
    fractions are reported; traffic = PMC HBM bytes per launch (profiles/pmc_gconv_wgrad3_<shape>.json, the
    rocprofv3 passes of tools/pmc_kernel.sh) averaged over the timed launches when every shape has one."""
    ms = sum(t for _, t, _ in gw)
    flop = sum(w["flop"] for _, _, w in gw)
    nbytes = sum(w["bytes"] for _, _, w in gw)
    mfma = flop / nbytes > RIDGE_FLOP_PER_BYTE
    tf = flop / (ms * 1e-3) / 1e12
    gbs = nbytes / (ms * 1e-3) / 1e9
    shapes = {}
    for _, t, w in gw:
        d = shapes.setdefault(w["shape"], [0.0, 0, w["flop"], w["bytes"]])
        d[0] += t
        d[1] += 1
    per, traffic = {}, None
    for sh in shapes:
        f = os.path.join(ROOT, "profiles", f"pmc_gconv_wgrad3_{sh.replace('->', 'to')}.json")
        if os.path.exists(f):
            with open(f) as fh:
                per[sh] = json.load(fh).get("hbm_bytes_per_launch")
    if per and all(per.get(w["shape"]) for _, _, w in gw):
        traffic = sum(per[w["shape"]] for _, _, w in gw) / len(gw)
    n_steps = max(1, round(len(gw) / 8))
    by = []
    for sh, (t, n, fl, nb) in sorted(shapes.items(), key=lambda kv: -kv[1][0]):
        a_us = 1e3 * t / n
        m2 = fl / nb > RIDGE_FLOP_PER_BYTE
        by.append({"shape": sh, "avg_us": round(a_us, 1), "launches_per_step": n / n_steps,
                   "bound": "mfma" if m2 else "hbm", "flop": fl, "bytes": nb,
                   "mfma_frac": round(fl / (a_us * 1e-6) / 1e12 / BF16_DENSE_PEAK_TFLOPS, 4),
                   "hbm_frac": round(nb / (a_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                   "pmc_hbm_bytes": per.get(sh)})
    return {"kernel": "gconv_wgrad3_kernel + gconv_wgrad3w_kernel (graph-conv weight gradient dWeff = dy^T x per "
                      "(joint, neighbour) pair, DMA-ring; the C = 256 launches run the 128 x 128 wide plan; the step's "
                      "largest kernel family in the rocprofv3 summary; 8 launches/step, bracketed alone by HIP events, "
                      "the slab reduction outside)",
            "rocprof_kernels": ["gconv_wgrad3_kernel", "gconv_wgrad3w_kernel"],
            "bound": "mfma" if mfma else "hbm", "achieved": round(tf if mfma else gbs, 2),
            "peak": BF16_DENSE_PEAK_TFLOPS if mfma else HBM_PEAK_GBS, "unit": "TFLOP/s" if mfma else "GB/s",
            "frac": round((tf / BF16_DENSE_PEAK_TFLOPS) if mfma else (gbs / HBM_PEAK_GBS), 4),
            "mfma_frac": round(tf / BF16_DENSE_PEAK_TFLOPS, 4), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
            "algorithmic_flop_per_launch": round(flop / len(gw)), "algorithmic_bytes_per_launch": round(nbytes / len(gw)),
            "traffic": traffic, "avg_launch_ms": round(ms / len(gw), 4), "launches_timed": len(gw), "by_shape": by}


def kernel_table(K, step, nsteps, top=4):
    """The step's kernels by time: every launch of the instrumented wrappers (native.KTIME_HOOK: temporal and
    1x1 convs, their weight gradients, graph conv fwd / data grad / weight grad + finish, BatchNorm apply and
    backward passes) bracketed by HIP events on its launch stream, over ``nsteps`` eager steps run after the
    timed region (recording ~150 event pairs per step costs host time, so not inside it).  Grouped by kernel
    family: time per step, algorithmic work per step (flops of the reference's formula for the GEMM-shaped
    families, bytes of the operands read + written once for the streaming ones), achieved rate and fraction of
    the roof the family's arithmetic intensity puts it under (MFMA above the ridge, HBM below)."""
    recs = []

    def hook(tag, phase, work):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream())
        recs.append((tag, phase, ev, work))

    K.KTIME_HOOK = hook
    try:
        for _ in range(nsteps):
            step()
        torch.cuda.synchronize()
    finally:
        K.KTIME_HOOK = None
    fam = {}
    open_ = {}
    for tag, phase, ev, work in recs:
        if phase == "start":
            open_[tag] = (ev, work)
            continue
        e0, w = open_.pop(tag)
        _, f, shape = tag.split(":", 2)
        d = fam.setdefault(f, {"ms": 0.0, "n": 0, "flop": 0.0, "bytes": 0.0, "shapes": {}})
        ms = e0.elapsed_time(ev)
        d["ms"] += ms
        d["n"] += 1
        d["flop"] += w["flop"] or 0.0
        d["bytes"] += w["bytes"] or 0.0
        s = d["shapes"].setdefault(shape, [0.0, 0, 0.0, 0.0])
        s[0] += ms
        s[1] += 1
        s[2] += w["flop"] or 0.0
        s[3] += w["bytes"] or 0.0

    def rate(ms, flop, nbytes):
        mfma = flop > 0 and flop / max(nbytes, 1.0) > RIDGE_FLOP_PER_BYTE
        if mfma:
            a = flop / (ms * 1e-3) / 1e12
            return "mfma", a, BF16_DENSE_PEAK_TFLOPS, "TFLOP/s"
        a = nbytes / (ms * 1e-3) / 1e9
        return "hbm", a, HBM_PEAK_GBS, "GB/s"

    out = []
    for f, d in sorted(fam.items(), key=lambda kv: -kv[1]["ms"])[:top]:
        bound, a, peak, unit = rate(d["ms"], d["flop"], d["bytes"])
        shapes = []
        for sh, (ms, n, fl, nb) in sorted(d["shapes"].items(), key=lambda kv: -kv[1][0]):
            b2, a2, p2, u2 = rate(ms, fl, nb)
            shapes.append({"shape": sh, "avg_us": round(1e3 * ms / n, 1), "launches_per_step": n / nsteps,
                           "bound": b2, "achieved": round(a2, 1), "unit": u2, "frac": round(a2 / p2, 4)})
        out.append({"kernel": f, "ms_per_step": round(d["ms"] / nsteps, 4), "launches_per_step": d["n"] / nsteps,
                    "bound": bound, "work_per_step": round((d["flop"] if bound == "mfma" else d["bytes"]) / nsteps),
                    "work_unit": "flop" if bound == "mfma" else "byte", "achieved": round(a, 1), "peak": peak,
                    "unit": unit, "frac": round(a / peak, 4), "by_shape": shapes})
    return {"method": f"HIP events around every instrumented launch, {nsteps} eager steps after the timed region",
            "top": out}


def cpu_baseline(pkg, model_cpu_sd):
    """Oracle (CPU restatement, oracle/stgcn_oracle.py) fwd+bwd on a bounded sample of the workload."""
    from oracle import stgcn_oracle as O

    threads = torch.get_num_threads()
    n_sample = int(os.environ.get("STGCN_CPU_SAMPLE_N", "32"))
    arch = dict(ARCH, graph=pkg.PKU_MMD)
    sd = {k: v.detach().float().clone().requires_grad_(v.dtype.is_floating_point) for k, v in model_cpu_sd.items()}
    gen = torch.Generator().manual_seed(0)
    weight = 1 - torch.rand(CLASSES, generator=gen) / CLASSES

    def step(n):
        x = torch.randn(n, 3, T_LEN, V_J, generator=gen)
        labels = torch.randint(0, CLASSES, (1, n), generator=gen)
        y = O.stgcn_model(x, sd, arch)
        loss_fn(y, labels, weight).backward()

    step(2)  # warm-up (allocator, oneDNN primitives)
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        step(n_sample)
    dt = time.perf_counter() - t0
    value = reps * n_sample * T_LEN / dt
    out = {"value": value, "unit": "skeleton-frames/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
           "sample": f"oracle fwd+bwd (torch CPU fp32) of the same 9-layer model at N={n_sample} T={T_LEN} V=25, "
                     f"{reps} steps, {dt:.1f} s"}
    # tools/calibrate_cpu.py (build container): oracle time / reference time on one host, same shapes/threads
    cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if os.path.exists(cal):
        with open(cal) as f:
            c = json.load(f)
        r = c["ratio_oracle_over_reference"]
        out["calibration"] = {"ratio_oracle_over_reference": r, "measured_on": c["host_cpu"],
                              "threads": c["threads"], "reference_equivalent_value": round(value * r, 1)}
    return out


def trial_lengths(n_units, W=T_LEN, seg=N_BATCH, seed=2):
    """Config 4's synthetic trial lengths ~ U[4000, 8000] (seed 2), as many trials as n_units needs."""
    import random
    rng = random.Random(seed)
    out, units = [], 0
    while units < n_units:
        L = rng.randint(4000, 8000)
        out.append(L)
        units += (L + L % seg) // seg
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=250)  # >= 2 s timed, so utilisation sampling sees it
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--config", type=int, default=2, choices=(2, 4))
    ap.add_argument("--torch-adam", action="store_true", help="torch's fused Adam instead of the package's")
    ap.add_argument("--accum", type=int, default=8, help="config 4: micro-steps per optimizer step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-layer-roofline", action="store_true", help="skip the north_star layer timing (profiling)")
    ap.add_argument("--graph", action="store_true", help="config 2: replay the step as HIP graphs")
    ap.add_argument("--sync-bn", action="store_true",
                    help="N > 1: SyncBatchNorm statistics over the ranks (syncbn.py) instead of the reference's "
                         "per-replica DataParallel statistics (the default)")
    ap.add_argument("--kernel-steps", type=int, default=3,
                    help="eager steps after the timed region whose kernel-wrapper launches are timed one by one "
                         "(the `kernels` table); 0 = off")
    args = ap.parse_args()
    if args.config == 4 and args.graph:
        sys.exit("bench.py: --graph needs fixed shapes (config 2); config 4's units have 49-65 windows")

    # STGCN_BENCH_REHEARSE=1: the N > 1 path (spawn, DDP, barriers, max-over-ranks timing, the JSON line) with every
    # rank on GPU 0 over gloo — a one-GPU rehearsal of the multi-GPU bench; its numbers are not a measurement
    rehearse = os.environ.get("STGCN_BENCH_REHEARSE") == "1"
    ndev = torch.cuda.device_count()  # does not initialise HIP (safe before spawning the ranks)
    if ndev < args.gpus and not rehearse:
        sys.exit(f"bench.py: --gpus {args.gpus} needs {args.gpus} HIP devices, {ndev} visible")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if rehearse:  # (--graph: gloo cannot be captured, so the bucketed step then runs uncaptured)
        local = 0
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo" if rehearse else "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import __graft_entry__ as ge
    pkg = ge.load_package()
    K = pkg.native
    par = pkg.parallel

    torch.manual_seed(1538574472)  # config seed (stgcn_local.json optimizer.seed)
    model = pkg.MODELS["st-gcn"](rank=None, **dict(ARCH, graph=pkg.PKU_MMD))
    cpu_sd = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(dev).set_compute_dtype(args.dtype)
    params = [p for p in model.parameters() if p.requires_grad]
    train_model = model
    if args.sync_bn:
        if args.graph:
            sys.exit("bench.py: --sync-bn exchanges statistics inside the forward (eager DDP step only)")
        pkg.convert_sync_batchnorm(model)
    if world > 1 and not args.graph:
        train_model = par.ddp(model, dev)  # RCCL all-reduce in 4 MB buckets, overlapped with bwd
    elif world > 1:  # identical replicas (DistributedDataParallel's broadcast from rank 0)
        for p in params:
            torch.distributed.broadcast(p.data, 0)
    # the reference's optimizer (Adam, lr 5e-4, processor.py:579): the package's Adam is torch's update rule with
    # every parameter in ONE launch (csrc/adam.hip; test_gpu_optim.py); --torch-adam: torch's fused Adam
    opt = torch.optim.Adam(params, lr=5e-4, fused=True, capturable=args.graph) if args.torch_adam else \
        pkg.optim.Adam(params, lr=5e-4)
    gen_t = torch.Generator(device=dev).manual_seed(12345)
    class_dist = torch.rand(CLASSES, device=dev, generator=gen_t) + 0.5
    crit = pkg.loss.Loss(dev, class_dist)

    # live timing of the roofline kernel (ROOF_TAGS: temporal-conv forward of the C=128/256 layers): HIP events
    # on the stream the kernel is launched on, with each launch's algorithmic flops.  ROCm refuses timing
    # events inside a captured graph, so in graph mode the events bracket the launches of one eager step run
    # right after the timed region.
    events = []
    timing = {"on": False}

    def hook(tag, phase, work=None):
        if (tag not in ROOF_TAGS and tag != ROOF_KERNEL) or not timing["on"]:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream())
        events.append((tag, ev, work))

    K.EVENT_HOOK = hook
    frames_done = [0]

    if args.config == 2:
        gen = torch.Generator(device=dev).manual_seed(rank)
        x = torch.randn(N_BATCH, 3, T_LEN, V_J, device=dev, generator=gen)
        labels = torch.randint(0, CLASSES, (1, N_BATCH), device=dev, generator=gen)

        def fwd_loss():
            pred = train_model(x).permute(2, 1, 0)  # (1, classes, windows): WindowSegment.mask_segment
            ce, mse = crit(0, pred, labels)
            return ce + mse  # DDP / the flat all-reduce average over ranks: loss / batch_size (processor.py:538)

        def eager_step():
            opt.zero_grad(set_to_none=True)  # as the reference's optimizer.zero_grad() (set_to_none)
            fwd_loss().backward()
            opt.step()
            frames_done[0] += N_BATCH * T_LEN

        if args.graph:  # its first (eager) step all-reduces too: the replicas stay identical
            # N > 1: ONE graph per step with the per-bucket RCCL all-reduces captured inside it, each issued when its
            # 4 MB bucket's gradients are accumulated (overlapped with the rest of the backward, as DDP eagerly)
            gstep = par.GraphedStep(fwd_loss, params, opt, world, bucket_mb=4 if world > 1 else None,
                                    capture=not (rehearse and world > 1))

            def step():
                gstep()
                frames_done[0] += N_BATCH * T_LEN
        else:
            step = eager_step
        for _ in range(max(args.warmup, 2)):
            step()
        torch.cuda.synchronize()
    else:
        units = par.units_for_rank(par.segment_units(trial_lengths(world * (args.warmup + args.steps + 2)),
                                                     T_LEN, N_BATCH), world, rank)
        gen = torch.Generator(device=dev).manual_seed(100 + rank)
        caps, labs = {}, {}

        def capture(k, L):
            if k not in caps:  # padded capture (1, 3, L + W - 1, V), labels (1, L): resident in HBM
                caps[k] = torch.nn.functional.pad(torch.randn(1, 3, L, V_J, device=dev, generator=gen),
                                                  (0, 0, T_LEN - 1, 0))
                labs[k] = torch.randint(0, CLASSES, (1, L), device=dev, generator=gen)
            return caps[k], labs[k]

        lengths = trial_lengths(world * (args.warmup + args.steps + 2))
        for u in units[:args.warmup + args.steps + 2]:
            capture(u.trial, lengths[u.trial])
        it = iter(units)
        micro = [0]

        def step():
            u = next(it)
            cap, lab = caps[u.trial], labs[u.trial]
            last = (micro[0] + 1) % args.accum == 0
            with par.accumulate(train_model, last=last):
                pred = train_model(pkg.segment.WindowBatch(cap, u.n0, u.nw, T_LEN)).permute(2, 1, 0)
                ce, mse = crit(u.i, pred, lab[:, u.y0:u.y1])
                ((ce + mse) / u.count).backward()  # processor.py:392 (ce, mse / num_subsegments)
            if last:
                opt.step()
                opt.zero_grad(set_to_none=True)
            micro[0] += 1
            frames_done[0] += u.nw * T_LEN

        for _ in range(max(args.warmup, 2)):
            step()
        torch.cuda.synchronize()

    timing["on"] = not args.graph
    frames_done[0] = 0
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        # the roofline launches are bracketed on every ROOF_EVERY-th timed step (the 16 extra timing events of an
        # instrumented step cost ~43 us; measured: 7.523 vs 7.480 ms/step with and without them on one box)
        timing["on"] = not args.graph and k % ROOF_EVERY == 0
        K.EVENT_HOOK = hook if timing["on"] else None  # no hook: the wrappers take their unsplit launch paths
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    frames = frames_done[0]
    if args.graph:
        timing["on"] = True
        K.EVENT_HOOK = hook
        eager_step()
        torch.cuda.synchronize()
    timing["on"] = False
    K.EVENT_HOOK = None
    ktable = None
    if args.kernel_steps > 0 and args.config == 2:
        ktable = kernel_table(K, eager_step, args.kernel_steps)
    if world > 1:
        t = torch.tensor([elapsed, float(frames)], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t[:1], op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(t[1:], op=torch.distributed.ReduceOp.SUM)
        elapsed, frames = t[0].item(), t[1].item()

    # (start, end) event pairs of the roofline launches: achieved = their algorithmic work / their time
    pairs = [(events[i][0], events[i][1].elapsed_time(events[i + 1][1]), events[i][2])
             for i in range(0, len(events) - 1, 2)]
    kt = [p for p in pairs if p[0] in ROOF_TAGS]
    gw = [p for p in pairs if p[0] == ROOF_KERNEL]
    k_ms = sum(t for _, t, _ in kt) / len(kt) if kt else float("nan")
    achieved = sum(w for _, _, w in kt) / (sum(t for _, t, _ in kt) * 1e-3) / 1e12 if kt else None

    value = frames / elapsed
    if rank == 0:
        traffic = None
        # HBM bytes per launch from the PMC passes of each launch shape (tools/pmc_conv.sh), averaged over
        # the timed launches like `achieved`
        per = {}
        for g in ROOF_TAGS:
            pmc = os.path.join(ROOT, "profiles", f"pmc_{g}.json")
            if os.path.exists(pmc):
                with open(pmc) as f:
                    per[g] = json.load(f).get("hbm_bytes_per_launch")
        if kt and all(per.get(g) for g, _, _ in kt) and args.config == 2:
            traffic = sum(per[g] for g, _, _ in kt) / len(kt)
        roof = gwgrad_roofline(gw, world) if gw and args.config == 2 else None
        lay = world == 1 and not args.no_layer_roofline and args.config == 2
        lroof = layer_roofline(pkg, dev, norm="BatchNorm") if lay else None
        lroof_ln = layer_roofline(pkg, dev, norm="LayerNorm") if lay else None
        cpu = None
        if not args.no_cpu_baseline and world == 1 and args.config == 2:
            cpu = cpu_baseline(pkg, cpu_sd)
        if args.config == 2:
            workload = "config 2: as_is st-gcn (fcn_in + 9 StgcnLayer, BatchNorm, Kt=9), fwd + loss + bwd + Adam"
            metric = "skeleton-frames/sec/GPU (fwd+bwd), 10-layer ST-GCN N=64 T=300 V=25"
        else:
            workload = ("config 4: as_is st-gcn DDP training on long unequal trials (U[4000,8000] frames, seed 2), "
                        f"WindowSegment units of 64 windows x T=300 dealt round-robin to ranks, fwd + loss + bwd "
                        f"per unit, no_sync + Adam every {args.accum} units")
            metric = "skeleton-frames/sec (fwd+bwd), 10-layer ST-GCN DDP, long trials, windows of T=300 V=25"
        out = {
            "metric": metric,
            "value": round(value, 1), "unit": "skeleton-frames/s", "per_gpu": round(value / world, 1),
            "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (randn skeletons, random labels/class weights), random-init weights",
            "config": {"workload": workload, "global_batch": N_BATCH * world, "seq_len": T_LEN, "joints": V_J,
                       "parallelism": (f"dp{world}" if world > 1 else "single") + (
                           " (REHEARSAL: all ranks on GPU 0 over gloo, not a measurement)" if rehearse else ""),
                       "bn_stats": "sync (all ranks)" if args.sync_bn and world > 1 else "per-replica",
                       "launch": "eager" if not args.graph else (
                           "hip-graph replay (fwd+bwd | Adam)" if world == 1 else
                           "hip-graph replay (fwd+bwd with captured 4 MB bucket all-reduces + Adam, one graph)")},
            "roofline": roof,
            "roofline_tcn_fwd": {"kernel": "conv_wide_kernel<128,9,8,1,0,64> (persistent warp-specialised Kt=9 "
                                           "stride-1 temporal conv fwd of the C=128 and C=256 layers, 4 launches/step)",
                         "bound": "mfma", "achieved": round(achieved, 2) if achieved else None,
                         "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / BF16_DENSE_PEAK_TFLOPS, 4) if achieved else None,
                         "traffic": traffic, "avg_launch_ms": round(k_ms, 4), "launches_timed": len(kt)},
            "kernels": ktable,
            "layer_roofline": lroof,
            "layer_roofline_ln": lroof_ln,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()

"""Benchmark: skeleton-frames/sec (fwd+bwd) of the 10-layer ST-GCN (fcn_in + 9 StgcnLayers, as_is BN,
Kt=9) at N=64 T=300 V=25 (BASELINE.json config 2), bf16 MFMA path, synthetic data.

One step = forward of the whole model on one (64, 3, 300, 25) batch + the reference loss
(weighted CE + clamped temporal MSE, utils/loss.py:25-41, windows as the time axis like
WindowSegment.mask_segment) + backward + Adam step.  Inputs are resident in HBM before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W]
Kernels are launched eagerly from Python (the GPU stays busy: launch cost < kernel time); --graph
captures the step into HIP graphs (torch.cuda.CUDAGraph) and replays them instead.
N > 1: one process per GPU, DistributedDataParallel over RCCL (backend "nccl").  Under
torch.distributed.run (WORLD_SIZE set) the ranks are the launcher's; `python bench.py --gpus N` alone
starts `torch.distributed.run --nproc-per-node N` as a child process (before anything touches the GPU)
and exits with its status.  Each rank processes its own 64 consecutive windows of one synthetic trial
of N*64 windows (weak scaling); the loss is the trial's (parallel.exchange_shard: the boundary MSE pair
crosses ranks), so the gradient equals the single-process one up to per-replica BatchNorm statistics,
as in the reference's DataParallel.
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


# The roofline kernel: conv_wide_kernel<128,9,8,1,0,64>, the Kt=9 stride-1 temporal-conv forward of the
# C=128 (T=150) and C=256 (T=75) layers — the dominant kernel template of the step (with its data-grad
# twin <128,9,8,0>), 4 launches per step.  Algorithmic work per launch = 2*N*T*V*C*C*Kt.
ROOF_TAGS = {"tcn_fwd_c128": 2.0 * N_BATCH * (T_LEN // 2) * V_J * 128 * 128 * 9,
             "tcn_fwd_c256": 2.0 * N_BATCH * (T_LEN // 4) * V_J * 256 * 256 * 9}


# north_star layer: StgcnLayer 64 -> 64, stride 1, Kt=9, BN, identity residual at N=64 T=300 V=25.
# Algorithmic forward work: 2NTV*Cin*P*Cout (gcn) + 2NP*Cout*T*V^2 (A-mix, dense as the
# reference counts it) + 2NTV*Cout^2*Kt (tcn) = 51.79 GFLOP.
LAYER_FWD_FLOP = (2.0 * N_BATCH * T_LEN * V_J * 64 * 3 * 64 + 2.0 * N_BATCH * 3 * 64 * T_LEN * V_J * V_J
                  + 2.0 * N_BATCH * T_LEN * V_J * 64 * 64 * 9)


def layer_roofline(pkg, dev, reps=20, norm="BatchNorm"):
    """Layer-level roofline of the north_star layer's forward: the fused path (inference; BatchNorm: pass 1
    graph-conv statistics, the fused graph conv + BN1 + ReLU + temporal conv kernel, BN2 + residual + ReLU;
    LayerNorm: the whole layer as the one fused kernel) against the unfused training-path forward of the
    same layer, both timed with HIP events around every launch of the layer on the launch stream; plus the
    fused kernel's own launch time (events around that launch)."""
    K = pkg.native
    torch.manual_seed(0)
    A = torch.tensor(pkg.Graph(**pkg.PKU_MMD).A, dtype=torch.float32, device=dev)
    layer = pkg.StgcnLayer(64, 64, (9, V_J), A.shape[0], V_J, stride=1, normalization=norm).to(dev)
    pkg.set_compute_dtype(layer, "bf16")
    x = torch.randn(N_BATCH, 64, T_LEN, V_J, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    kev = []

    def hook(tag, phase):
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

    orig = K.layer_fused

    def tagged(*a, **k):
        k["tag"] = "layer_fused"
        return orig(*a, **k)

    K.layer_fused = tagged
    prev_hook = K.EVENT_HOOK
    K.EVENT_HOOK = hook
    prev_route = pkg.routing.ROUTING.fused_bn_inference
    pkg.routing.ROUTING.fused_bn_inference = True  # BatchNorm layers take the fused path on request only
    try:
        with torch.no_grad():
            fused_ms = timed(lambda: layer(x, A))
    finally:
        K.layer_fused = orig
        K.EVENT_HOOK = prev_hook
        pkg.routing.ROUTING.fused_bn_inference = prev_route
    xg = x.detach().requires_grad_(True)  # a differentiable input: the training path's forward (unfused)
    unfused_ms = timed(lambda: layer(xg, A))
    pairs = [(kev[i], kev[i + 1]) for i in range(6, len(kev) - 1, 2)]  # skip the warm-up launches
    k_ms = sum(a.elapsed_time(b) for a, b in pairs) / len(pairs) if pairs else None
    achieved = LAYER_FWD_FLOP / (fused_ms * 1e-3) / 1e12
    return {"layer": f"StgcnLayer(64, 64, (9, 25), 3, 25, {norm}) forward, N=64 T=300 V=25, bf16 (north_star)",
            "bound": "mfma", "algorithmic_gflop": round(LAYER_FWD_FLOP / 1e9, 2),
            "fused_fwd_ms": round(fused_ms, 4), "unfused_fwd_ms": round(unfused_ms, 4),
            "fused_kernel_ms": round(k_ms, 4) if k_ms else None,
            "achieved": round(achieved, 2), "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / BF16_DENSE_PEAK_TFLOPS, 4),
            "unfused_frac": round(LAYER_FWD_FLOP / (unfused_ms * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS, 4)}


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=250)  # >= 2 s timed, so utilisation sampling sees it
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-layer-roofline", action="store_true", help="skip the north_star layer timing (profiling)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the step into HIP graphs and replay them (measured slower than eager here)")
    args = ap.parse_args()

    ndev = torch.cuda.device_count()  # does not initialise HIP (safe before spawning the ranks)
    if ndev < args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} needs {args.gpus} HIP devices, {ndev} visible")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import __graft_entry__ as ge
    pkg = ge.load_package()
    K = pkg.native

    torch.manual_seed(1538574472)  # config seed (stgcn_local.json optimizer.seed)
    model = pkg.MODELS["st-gcn"](rank=None, **dict(ARCH, graph=pkg.PKU_MMD))
    cpu_sd = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(dev).set_compute_dtype(args.dtype)
    params = [p for p in model.parameters() if p.requires_grad]
    train_model = model
    if world > 1 and not args.graph:
        train_model = pkg.parallel.ddp(model, dev, bucket_cap_mb=16)  # RCCL all-reduce overlapped with bwd
    elif world > 1:  # identical replicas (DistributedDataParallel's broadcast from rank 0)
        for p in params:
            torch.distributed.broadcast(p.data, 0)
    # the reference's optimizer (Adam, lr 5e-4); the fused multi-tensor implementation is the same update
    # rule in one launch per parameter chunk instead of one foreach launch per elementwise op
    opt = torch.optim.Adam(params, lr=5e-4, fused=True, capturable=args.graph)

    gen = torch.Generator(device=dev).manual_seed(rank)
    x = torch.randn(N_BATCH, 3, T_LEN, V_J, device=dev, generator=gen)
    # the trial's labels and class distribution are the same on every rank (seeded alike)
    gen_t = torch.Generator(device=dev).manual_seed(12345)
    labels_trial = torch.randint(0, CLASSES, (1, N_BATCH * world), device=dev, generator=gen_t)
    class_dist = torch.rand(CLASSES, device=dev, generator=gen_t) + 0.5
    crit = pkg.loss.Loss(dev, class_dist)
    w0, w1 = rank * N_BATCH, (rank + 1) * N_BATCH
    labels = labels_trial[:, w0:w1]

    # Gradient exchange (N > 1): eager mode uses DistributedDataParallel (RCCL all-reduce of 16 MB
    # buckets overlapped with backward); graph mode all-reduces one flat fp32 buffer between the
    # backward graph and the optimizer graph.  BatchNorm statistics stay per replica in both.
    numels = [p.numel() for p in params]
    flat = torch.zeros(sum(numels), device=dev) if world > 1 and args.graph else None

    def fwd_bwd():
        pred = train_model(x).permute(2, 1, 0)  # (1, classes, windows): WindowSegment.mask_segment
        shard = pkg.parallel.exchange_shard(pred, labels_trial, crit.weight, w0, N_BATCH * world) \
            if world > 1 else None
        ce, mse = crit(0, pred, labels, shard=shard)
        loss = (ce + mse) * world  # DDP averages over ranks; the shares sum to the trial's loss
        loss.backward()
        if flat is not None:
            torch.cat([p.grad.reshape(-1) for p in params], out=flat)
        return loss

    def opt_step():
        if flat is not None:
            for p, g in zip(params, torch.split(flat, numels)):
                p.grad.copy_(g.view_as(p.grad)).div_(world)
        opt.step()

    def eager_step():
        opt.zero_grad(set_to_none=flat is None)  # as the reference's optimizer.zero_grad() (set_to_none)
        fwd_bwd()
        if flat is not None:
            torch.distributed.all_reduce(flat)
        opt_step()

    # live timing of the roofline kernel (ROOF_TAGS: temporal-conv forward of the C=128/256 layers): HIP events on
    # the stream the kernel is launched on.  ROCm refuses timing events inside a captured graph, so in
    # graph mode the events bracket the launches of one eager step run right after the timed region.
    events = []
    timing = {"on": False}

    def hook(tag, phase):
        if tag not in ROOF_TAGS or not timing["on"]:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream())
        events.append((tag, ev))

    K.EVENT_HOOK = hook
    for _ in range(max(args.warmup, 2)):
        eager_step()
    torch.cuda.synchronize()

    graphs = None
    if args.graph:
        # capture: [zero grads, fwd, loss, bwd (+ flatten)] and [unflatten/average, Adam]; grads keep
        # their addresses, so replays overwrite them in place
        opt.zero_grad(set_to_none=False)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):
                for p in params:
                    p.grad.zero_()
                fwd_bwd()
            with torch.cuda.graph(g2):
                opt_step()
        torch.cuda.current_stream().wait_stream(s)
        graphs = (g1, g2)

        def step():
            g1.replay()
            if flat is not None:
                torch.distributed.all_reduce(flat)
            g2.replay()
        for _ in range(2):
            step()
    else:
        step = eager_step

    if not args.graph:
        timing["on"] = True
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if args.graph:
        timing["on"] = True
        eager_step()
        torch.cuda.synchronize()
    timing["on"] = False
    K.EVENT_HOOK = None
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()

    # eager mode: every launch of the timed region; graph mode: the 6 launches of the step after it
    # (start, end) event pairs of the roofline launches: achieved = their algorithmic flops / their time
    kt = [(events[i][0], events[i][1].elapsed_time(events[i + 1][1])) for i in range(0, len(events) - 1, 2)]
    k_ms = sum(t for _, t in kt) / len(kt) if kt else float("nan")
    achieved = sum(ROOF_TAGS[g] for g, _ in kt) / (sum(t for _, t in kt) * 1e-3) / 1e12 if kt else None

    frames = world * args.steps * N_BATCH * T_LEN
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
        if kt and all(per.get(g) for g, _ in kt):
            traffic = sum(per[g] for g, _ in kt) / len(kt)
        lay = world == 1 and not args.no_layer_roofline
        lroof = layer_roofline(pkg, dev) if lay else None
        lroof_ln = layer_roofline(pkg, dev, norm="LayerNorm") if lay else None
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(pkg, cpu_sd)
        out = {
            "metric": "skeleton-frames/sec/GPU (fwd+bwd), 10-layer ST-GCN N=64 T=300 V=25",
            "value": round(value, 1), "unit": "skeleton-frames/s", "per_gpu": round(value / world, 1),
            "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (randn skeletons, random labels/class weights), random-init weights",
            "config": {"workload": "config 2: as_is st-gcn (fcn_in + 9 StgcnLayer, BatchNorm, Kt=9), fwd + loss + "
                                   "bwd + Adam", "global_batch": N_BATCH * world, "seq_len": T_LEN, "joints": V_J,
                       "parallelism": f"dp{world}" if world > 1 else "single",
                       "launch": "eager" if not args.graph else "hip-graph replay (fwd+bwd | allreduce | Adam)"},
            "roofline": {"kernel": "conv_wide_kernel<128,9,8,1,0,64> (persistent warp-specialised Kt=9 stride-1 "
                                   "temporal conv fwd of the C=128 and C=256 layers, 4 launches/step)",
                         "bound": "mfma", "achieved": round(achieved, 2) if achieved else None,
                         "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / BF16_DENSE_PEAK_TFLOPS, 4) if achieved else None,
                         "traffic": traffic, "avg_launch_ms": round(k_ms, 4), "launches_timed": len(kt)},
            "layer_roofline": lroof,
            "layer_roofline_ln": lroof_ln,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    del graphs
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()

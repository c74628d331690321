"""Per-phase cycle accounts of the one-launch RT frame kernel (stgcn_rt_frame) from a -DSTGCN_RT_PROF=1 build:
    make -C realtime-st-gcn_amd/csrc BUILD=../build_p LIBDIR=../lib_p DEFS=-DSTGCN_RT_PROF=1
    STGCN_LIB=$PWD/realtime-st-gcn_amd/lib_p/libstgcn_amd.so python tools/rt_prof.py [blocks]
Runs config 3 (tools/bench_configs.py's model) for a few frames, then prints per layer the mean (over workgroups)
of the cycles worker thread 64 spent in each phase of the last frame, and the spread of barrier exits."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_configs import RT_ARCH  # noqa: E402

PH = ["conv", "mix+drain", "prefetch", "barrier", "a loads", "LN stats", "y"]

if __name__ == "__main__":
    P = ge.load_package()
    dev = torch.device("cuda", 0)
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    torch.manual_seed(0)
    m = P.MODELS["rt-st-gcn"](rank=None, **dict(RT_ARCH, graph=P.PKU_MMD)).to(dev).eval()
    m.prepare_benchmark(RT_ARCH)
    x = torch.randn(1, 3, 1, 25, device=dev)
    with torch.no_grad():
        m(x)
        if G:
            m._frame_pack[1][0].blocks = G
        for _ in range(20):
            m(x)
    torch.cuda.synchronize()
    Gr = G or 64
    L = len(m.st_gcn)
    lib = P._lib.lib()
    fn = lib.stgcn_rt_prof
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_long]
    n = 256 * 12 * 8
    buf = np.zeros(n, dtype=np.int64)
    if fn(buf.ctypes.data, n) != 0:
        raise SystemExit("not a profiling build (-DSTGCN_RT_PROF=1)")
    a = buf.reshape(256, 12, 8)[:Gr, :L].astype(np.float64)
    t0 = a[:, 0, 0].min()
    tot = a[:, L - 1, 7].max() - t0
    print(f"workgroups {Gr}, frame {tot:.0f} cycles (thread 64 stamps, s_memtime)")
    print("layer " + " ".join(f"{p:>9s}" for p in PH) + "   exit-spread")
    for l in range(L):
        d = np.diff(a[:, l, :], axis=1).mean(axis=0)
        spread = a[:, l, 4].max() - a[:, l, 4].min()
        print(f"{l:5d} " + " ".join(f"{v:9.0f}" for v in d) + f"   {spread:9.0f}")
    gaps = [(a[:, l + 1, 0] - a[:, l, 7]).mean() for l in range(L - 1)]
    print("between layers (stage of next task):", " ".join(f"{g:.0f}" for g in gaps))

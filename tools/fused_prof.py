"""Per-wave cycle accounts of the fused layer kernel (a -DSTGCN_FUSED_DBG=1024 build, pointed at by STGCN_LIB):
runs the north_star layer's LayerNorm fused forward a few times, reads g_fused_prof and prints, per role, the
mean cycles per block spent in each phase (GCN: DMA wait, compute, barrier; TCN: k-loop, epilogue, barrier).

    STGCN_LIB=$PWD/realtime-st-gcn_amd/lib_p/libstgcn_amd.so python tools/fused_prof.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

if __name__ == "__main__":
    pkg = ge.load_package()
    dev = torch.device("cuda", 0)
    norm = "LayerNorm"
    bench.layer_roofline(pkg, dev, reps=3, norm=norm)
    torch.cuda.synchronize()
    lib = pkg._lib.lib()
    fn = lib.stgcn_fused_prof
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_long]
    n = 256 * 8 * 6
    buf = np.zeros(n, dtype=np.int64)
    if fn(buf.ctypes.data, n) != 0:
        raise SystemExit("not a profiling build (STGCN_FUSED_DBG & 1024)")
    a = buf.reshape(256, 8, 6).astype(np.float64)
    tcn, gcn = a[:, :4], a[:, 4:]
    print(f"total cycles per wave: mean {a[:, :, 3].mean():.0f} (max {a[:, :, 3].max():.0f})")
    m = tcn.mean(axis=(0, 1))
    print(f"TCN waves: k-loop {m[0]:.0f}  z stores (LN: normalise + stores) {m[4]:.0f}  BN2 partials (LN: statistics) "
          f"{m[1]:.0f}  LN hand-off {m[5]:.0f}  barrier {m[2]:.0f}")
    g = gcn.mean(axis=(0, 1))
    print(f"GCN waves: DMA wait {g[0]:.0f}  compute (round 6: the matrix part) {g[1]:.0f}  epilogue {g[4]:.0f}  "
          f"barrier {g[2]:.0f}")

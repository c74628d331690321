"""Per-wave cycle accounts of the temporal-conv weight-gradient ring kernel (a -DWR_PROF=1 build, pointed at by
STGCN_LIB): runs the C = 64 (or given) config-2 shape once and prints the mean cycles per wave of each phase of the
step loop (vmcnt wait, barrier wait, DMA issue + transform, compute) for waves 0-3 and 4-7.
    STGCN_LIB=$PWD/realtime-st-gcn_amd/lib_p/libstgcn_amd.so python tools/wr_prof.py [C] [pro]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 64
pro = int(sys.argv[2]) if len(sys.argv) > 2 else 1
pkg = ge.load_package()
K = pkg.native
dev = "cuda:0"
N, V, T = 64, 25, 300 if C == 64 else 150
x = torch.randn(N, C, T, V, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
dy = torch.randn(N, C, T, V, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
kw = dict(Kt=9, stride=1, pad=4, pro=pro, pro_a=sc if pro else None, pro_b=sh if pro else None)
for _ in range(3):
    K.conv_wgrad_w(x, dy, C, C, T, T, **kw)
torch.cuda.synchronize()
lib = pkg._lib.lib()
fn = lib.stgcn_wr_prof
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_long]
buf = np.zeros(256 * 8 * 5, dtype=np.int64)
if fn(buf.ctypes.data, buf.size) != 0:
    raise SystemExit("not a profiling build (-DWR_PROF=1)")
a = buf.reshape(256, 8, 5).astype(np.float64)
for name, sl in (("waves 0-3", slice(0, 4)), ("waves 4-7", slice(4, 8))):
    m = a[:, sl].mean(axis=(0, 1))
    print(f"{name}: vmcnt wait {m[0]:.0f}  barrier {m[1]:.0f}  issue+transform {m[2]:.0f}  compute {m[3]:.0f}  "
          f"total {m[4]:.0f} cycles (max total {a[:, sl, 4].max():.0f})")

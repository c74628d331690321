"""Phase timers of conv_wide.hip (STGCN_WIDE_DBG=4): per block, s_memtime cycles of MMA wave 0
(k-step compute, E-barrier wait, tile-end dump, I-barrier wait) and helper wave 4 (drain, halo store,
halo load issue, E wait, I wait).   python tools/wide_timers.py [case ...]"""
import ctypes
import os
import sys

import numpy as np
import torch

os.environ["STGCN_WIDE_DBG"] = "4"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

P = ge.load_package()
K = P.native
dev = "cuda:0"
dt = torch.bfloat16
CASES = {"tcn_fwd_c128": (64, 150, 25, 128, 128, False, 1), "tcn_fwd_c256": (64, 75, 25, 256, 256, False, 1),
         "tcn_dgrad_c128": (64, 150, 25, 128, 128, True, 0)}
lib = ctypes.CDLL(P._lib.LIB_PATH)
for name in (sys.argv[1:] or list(CASES)):
    N, T, V, Cin, Cout, trans, pro = CASES[name]
    x = torch.randn(N, Cin, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    wp, cp, kp = K.pack_weight(torch.randn(9, Cout, Cin, device=dev) * 0.05, dt)
    kw = dict(pro=1, pro_a=torch.rand(Cin, device=dev) + 0.5, pro_b=torch.randn(Cin, device=dev)) if pro else {}
    if not trans:
        kw["stats"] = torch.zeros((K.row_blocks(N * T * V, Cout), cp, 4), device=dev)
    f = lambda: K.conv_rows(x, wp, Cin, Cout, cp, kp, T, T, Kt=9, pad=4, trans=trans, **kw)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    f()
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros(16 * 4096, dtype=np.int64)
    assert lib.stgcn_debug_wide_timers(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(buf.size)) == 0
    d = buf.reshape(-1, 16)
    d = d[d[:, 0] > 0]
    m = d.mean(axis=0)
    print(f"{name:16s} {e0.elapsed_time(e1) * 1e3:7.1f} us  blocks {len(d)}\n"
          f"   MMA    compute {m[0]:8.0f}  E-wait {m[4] - m[3]:7.0f}  (k-steps incl {m[3]:.0f})  dump {m[1]:6.0f}  I-wait {m[2]:6.0f}\n"
          f"   helper drain+wait {m[8]:7.0f}  store {m[9]:7.0f}  issue {m[10]:6.0f}  E-wait {m[11]:7.0f}  I-wait {m[12]:6.0f}"
          f"  tail {m[13]:6.0f}", flush=True)

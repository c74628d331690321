"""Phase timers of the frame-tiled conv (STGCN_TILE_DBG=1): per block (wave 0), s_memtime cycles spent
issuing the next chunk's loads, in the MFMA loop, staging the next A halo (incl. its vmcnt wait) and at
the chunk barrier, plus the whole kernel.   python tools/tile_dbg.py [case ...]"""
import ctypes
import os
import sys

import numpy as np
import torch

os.environ["STGCN_TILE_DBG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

P = ge.load_package()
K = P.native
dev = "cuda:0"
dt = torch.bfloat16
CASES = {  # N, T, V, Cin, Cout, Kt, stride, trans, pro
    "tcn_fwd_c128": (64, 150, 25, 128, 128, 9, 1, False, 1),
    "tcn_fwd_c256": (64, 75, 25, 256, 256, 9, 1, False, 1),
    "tcn_dgrad_c256": (64, 75, 25, 256, 256, 9, 1, True, 0),
    "tcn_fwd_s2_c128": (64, 300, 25, 128, 128, 9, 2, False, 1),
}
lib = ctypes.CDLL(P._lib.LIB_PATH)
for name in (sys.argv[1:] or list(CASES)):
    N, T, V, Cin, Cout, Kt, s, trans, pro = CASES[name]
    pad = (Kt - 1) // 2
    T_out = T if s == 1 else (T - 1) // s + 1
    Ti, To = (T_out, T) if trans else (T, T_out)
    x = torch.randn(N, Cin, Ti, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
    w = torch.randn(Kt, Cout, Cin, device=dev) * 0.05
    wp, cp, kp = K.pack_weight(w, dt)
    kw = dict(pro=1, pro_a=torch.rand(Cin, device=dev) + 0.5, pro_b=torch.randn(Cin, device=dev)) if pro else {}
    if not trans:
        kw["stats"] = torch.zeros((K.row_blocks(N * To * V, Cout), cp, 4), device=dev)
    f = lambda: K.conv_rows(x, wp, Cin, Cout, cp, kp, Ti, To, Kt=Kt, stride=s, pad=pad, trans=trans,
                            bias=torch.randn(Cout, device=dev), **kw)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    f()
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros(8 * 8192, dtype=np.int64)
    assert lib.stgcn_debug_tile_timers(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(buf.size)) == 0
    d = buf.reshape(-1, 8)
    d = d[d[:, 5] > 0]
    m = d.mean(axis=0)
    print(f"{name:18s} {e0.elapsed_time(e1) * 1e3:7.1f} us  blocks {len(d)}  chunks {m[5]:.0f}  per block: "
          f"load-issue {m[0]:.0f}  mfma {m[1]:.0f}  stage {m[2]:.0f}  barrier {m[3]:.0f}  total {m[4]:.0f} cycles"
          f"  (per chunk: {m[0] / m[5]:.0f} / {m[1] / m[5]:.0f} / {m[2] / m[5]:.0f} / {m[3] / m[5]:.0f})", flush=True)

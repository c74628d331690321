"""Phase timers of the persistent C=64 conv (STGCN_PERSIST_DBG=1 build path): per block, for the
group-0 and group-1 lead waves, s_memtime cycles in compute / VALU phases / barriers."""
import ctypes
import os
import sys

import numpy as np
import torch

os.environ["STGCN_PERSIST_DBG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

P = ge.load_package()
K = P.native
dev = "cuda:0"
dt = torch.bfloat16
N, T, V, C = 64, 300, 25, 64
x = torch.randn(N, C, T, V, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
w = torch.randn(9, C, C, device=dev) * 0.05
wp, cp, kp = K.pack_weight(w, dt)
sc = torch.rand(C, device=dev) + 0.5
sh = torch.randn(C, device=dev)
b = torch.randn(C, device=dev)
st = torch.zeros((K.row_blocks(N * T * V, C), cp, 4), device=dev)
for _ in range(3):
    K.conv_rows(x, wp, C, C, cp, kp, T, T, Kt=9, pad=4, bias=b, pro=1, pro_a=sc, pro_b=sh, stats=st)
torch.cuda.synchronize()
lib = ctypes.CDLL(P._lib.LIB_PATH)
buf = np.zeros(8 * 256, dtype=np.int64)
assert lib.stgcn_debug_persist_timers(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(buf.size)) == 0
d = buf.reshape(256, 2, 4)
for gi in range(2):
    print("group %d: compute %.0f  epilogue %.0f  commit %.0f  prefetch %.0f  (mean cycles per block)" %
          (gi, d[:, gi, 0].mean(), d[:, gi, 1].mean(), d[:, gi, 2].mean(), d[:, gi, 3].mean()))

"""Tensor-level wrappers over the C-ABI (one function per entry point of include/stgcn_amd.h).

Activations are torch tensors whose memory is channels-last rows: either logical (N, C, T, V)
tensors in ``torch.channels_last`` format or plain contiguous (N, T, V, C) buffers.  Every
wrapper only validates, extracts raw pointers/strides and calls the library on the current
HIP stream; all arithmetic happens in the HIP kernels.
"""
from __future__ import annotations


import ctypes

import torch

from . import _lib as L
from .routing import ROUTING

class device_of:
    """Device guard (SURVEY 8(b) threading): make the device of tensor ``t`` current for the body, so that
    L.stream() — the current stream of the current device — and every allocation belong to the tensor's
    device even when the caller has another device current (DataParallel-style threads, multi-GPU hosts).
    Costs one device query when the device is already current."""
    __slots__ = ("idx", "prev")

    def __init__(self, t):
        self.idx = t.device.index if getattr(t, "is_cuda", False) else None
        self.prev = None

    def __enter__(self):
        if self.idx is not None:
            cur = torch._C._cuda_getDevice()
            if cur != self.idx:
                torch._C._cuda_setDevice(self.idx)
                self.prev = cur
        return self

    def __exit__(self, *exc):
        if self.prev is not None:
            torch._C._cuda_setDevice(self.prev)
            self.prev = None
        return False


def on_tensor_device(cls):
    """Class decorator for the autograd Functions: run forward / backward under device_of(the first CUDA
    tensor argument)."""
    import functools

    def wrap(fn):
        @functools.wraps(fn)
        def g(ctx, *args):
            t = next((a for a in args if isinstance(a, torch.Tensor) and a.is_cuda), None)
            if t is None:
                return fn(ctx, *args)
            with device_of(t):
                return fn(ctx, *args)
        return staticmethod(g)

    for name in ("forward", "backward"):
        if name in cls.__dict__:
            setattr(cls, name, wrap(cls.__dict__[name].__func__))
    return cls


# Optional instrumentation: callable(tag, phase, work) invoked right before ("start", with the launch's
# algorithmic flops where the wrapper knows them, else None) and after ("end", None) a tagged launch, on the
# launching stream (bench.py records HIP events with it).  None = off.
EVENT_HOOK = None
# Per-kernel timing: callable(tag, phase, work) for EVERY launch of the instrumented wrappers (conv_rows,
# conv_wgrad_w, gconv, gconv_wgrad(_finish), bn_apply, the fused BN backward), tag "k:<family>:<shape>", work
# {"flop", "bytes"} (algorithmic).  bench.py's kernel table installs it outside its timed region.  None = off.
KTIME_HOOK = None


def _k_start(h, family, shape, flop=None, nbytes=None):
    """Report a kernel-wrapper launch to the hook ``h`` (= KTIME_HOOK, checked by the caller so that the
    uninstrumented path costs one global read): tag ``"k:<family>:<shape>"``, work ``{"flop": algorithmic
    flops, "bytes": algorithmic HBM bytes}`` — bench.py's per-kernel table.  Returns the tag for _k_end."""
    tag = f"k:{family}:{shape}"
    h(tag, "start", {"flop": flop, "bytes": nbytes})
    return tag


def _dense(A: torch.Tensor) -> torch.Tensor:
    """Adjacency as the C-ABI reads it: dense row-major fp32 (graph.py's A is a transposed numpy view, and
    torch.tensor keeps those strides)."""
    return A if (A.dtype == torch.float32 and A.is_contiguous()) else A.float().contiguous()


def rows_ld(t: torch.Tensor) -> int:
    """Row stride (elements) of a logical (N,C,T,V) activation stored channels-last."""
    if t.dim() != 4 or (t.stride(1) != 1 and t.shape[1] > 1):
        raise RuntimeError(f"stgcn_amd: expected a channels-last (N,C,T,V) activation, strides {t.stride()}")
    N, C, T, V = t.shape
    if V > 1:
        ld = t.stride(3)
        if T > 1 and t.stride(2) != V * ld:
            raise RuntimeError("stgcn_amd: activation rows are not evenly strided")
        if N > 1 and t.stride(0) != T * V * ld:
            raise RuntimeError("stgcn_amd: activation rows are not evenly strided")
        return ld
    if T > 1:
        return t.stride(2)
    return t.stride(0) if N > 1 else C


def cl_empty(N, C, T, V, dtype, device):
    """Logical (N,C,T,V) tensor with channels-last (rows) memory."""
    return torch.empty((N, T, V, C), dtype=dtype, device=device).permute(0, 3, 1, 2)


def to_rows(x: torch.Tensor, dtype) -> torch.Tensor:
    """Make ``x`` (N,C,T,V) a channels-last tensor of ``dtype`` (no copy if already)."""
    L.require_device(x)
    if x.dtype != dtype:
        x = x.to(dtype)
    if not (x.stride(1) == 1 and x.is_contiguous(memory_format=torch.channels_last)):
        x = x.contiguous(memory_format=torch.channels_last)
    return x


def col_tile(cout: int) -> int:
    return L.lib().stgcn_conv_rows_col_tile(cout)


def row_blocks(M: int, cout: int) -> int:
    return L.lib().stgcn_conv_rows_row_blocks(M, cout)


def pack_weight(w3: torch.Tensor, dtype, stride: int = 1, trans: bool = False, plan=None) -> tuple:
    """[Kt][Cout][Cin] float weight -> padded contiguous [Kt][Cout_pad][Cin_pad] of ``dtype``.

    bf16 Kt=9 weights with >= 128 (padded) channels on both sides also get the MFMA-fragment image the
    wide-channel conv kernel reads (stgcn_pack_weight_frag), in the same allocation; ``out.frag_ptr``
    is its address and ``out.frag_stride`` the conv stride it is for (conv_rows passes it as ``w_frag``
    to calls of that stride).  For ``stride=2`` the image is the parity-folded 5-tap form
    (stgcn_pack_weight_s2frag, ``trans`` selecting the data-gradient fold).
    ``plan`` (a PrepPlan): allocate the same buffers but only record the jobs; PrepPlan.run() fills them
    (with every other pack of the model) in one launch."""
    Kt, Co, Ci = w3.shape
    cp = -(-Co // col_tile(Co)) * col_tile(Co)
    kp = -(-Ci // 32) * 32
    if w3.dtype != torch.float32:
        w3 = w3.float()
    s0, s1, s2 = w3.stride()
    n = Kt * cp * kp
    code = L.dtype_code(dtype)
    if dtype == torch.bfloat16 and Kt == 9 and stride == 2 and Co % 64 == 0 and Ci % 64 == 0:
        nf = 5 * 2 * Co * Ci
        buf = torch.empty(n + nf, dtype=dtype, device=w3.device)
        out = buf[:n].view(Kt, cp, kp)
        if plan is not None:
            plan.add(kind=0, dtype=code, src=w3, Kt=Kt, Co=Co, Ci=Ci, cp=cp, kp=kp, dst=out)
            plan.add(kind=1, dtype=code, src=w3, Co=Co, Ci=Ci, trans=int(trans), dst=buf[n:])
        else:
            L.check(L.lib().stgcn_pack_weight(w3.data_ptr(), s0, s1, s2, Kt, Co, Ci, out.data_ptr(), cp, kp,
                                              code, L.stream()), "pack_weight")
            L.check(L.lib().stgcn_pack_weight_s2frag(w3.data_ptr(), s0, s1, s2, Co, Ci, buf[n:].data_ptr(),
                                                     int(trans), code, L.stream()), "pack_weight_s2frag")
        out.frag_ptr, out.frag_stride = buf[n:].data_ptr(), 2
        return out, cp, kp
    frag = None
    if dtype == torch.bfloat16 and Kt == 9 and stride == 1 and cp % 64 == 0 and kp % 64 == 0:
        frag = 1
    elif dtype == torch.bfloat16 and Kt == 1 and kp == Ci and Ci in (64, 128, 192, 256) and Co % 64 == 0:
        frag = 0  # 1x1 weights: fragment image for the row-GEMM kernel (conv1x1.hip), valid at any stride
    if frag is not None:
        buf = torch.empty(2 * n, dtype=dtype, device=w3.device)
        out = buf[:n].view(Kt, cp, kp)
        if plan is not None:
            plan.add(kind=0, dtype=code, src=w3, Kt=Kt, Co=Co, Ci=Ci, cp=cp, kp=kp, dst=out, dst_frag=buf[n:])
        else:
            L.check(L.lib().stgcn_pack_weight_frag(w3.data_ptr(), s0, s1, s2, Kt, Co, Ci, out.data_ptr(),
                                                   buf[n:].data_ptr(), cp, kp, code, L.stream()), "pack_weight_frag")
        out.frag_ptr, out.frag_stride = buf[n:].data_ptr(), frag
        return out, cp, kp
    out = torch.empty((Kt, cp, kp), dtype=dtype, device=w3.device)
    if plan is not None:
        plan.add(kind=0, dtype=code, src=w3, Kt=Kt, Co=Co, Ci=Ci, cp=cp, kp=kp, dst=out)
    else:
        L.check(L.lib().stgcn_pack_weight(w3.data_ptr(), s0, s1, s2, Kt, Co, Ci, out.data_ptr(), cp, kp,
                                          code, L.stream()), "pack_weight")
    return out, cp, kp


class PrepPlan:
    """Every packed operand of a model's training step, prepared by ONE launch (stgcn_prep_run): the jobs
    pack_weight / gconv_weights would launch one by one are recorded once (their output buffers are
    allocated here and stay put), the job table is validated (stgcn_prep_check) and uploaded once, and
    run() re-fills every buffer from the current parameter values.  ``key`` identifies the parameter
    storages the jobs read; the owner rebuilds the plan when it changes (e.g. after .to())."""

    def __init__(self, device, key=None):
        self.device = device
        self.key = key
        self._jobs = []
        self._keep = []  # sources and outputs: the table holds raw pointers into them
        self._table = self._starts = None
        self.nblocks = 0

    def add(self, kind, dtype, src, dst, Kt=1, Co=0, Ci=0, cp=0, kp=0, dst_frag=None, trans=0, A=None, M=None,
            nbr=None, deg=None, P=0, V=0, J=0, R_pad=0, C_pad=0, bconv=None, bias2d=None):
        if self._table is not None:
            raise RuntimeError("stgcn_amd: PrepPlan is finalized")
        j = L.PrepJob()
        j.kind, j.dtype, j.trans, j.Kt, j.Co, j.Ci, j.cp, j.kp = kind, dtype, int(trans), Kt, Co, Ci, cp, kp
        j.s0, j.s1, j.s2 = src.stride() if src.dim() == 3 else (0,) + tuple(src.stride())
        j.src, j.dst, j.dst_frag = src.data_ptr(), dst.data_ptr(), L.ptr(dst_frag)
        j.A, j.M, j.nbr, j.deg, j.bconv, j.bias2d = L.ptr(A), L.ptr(M), L.ptr(nbr), L.ptr(deg), L.ptr(bconv), \
            L.ptr(bias2d)
        j.P, j.V, j.J, j.R_pad, j.C_pad = P, V, J, R_pad, C_pad
        self._jobs.append(j)
        self._keep += [t for t in (src, dst, dst_frag, A, M, nbr, deg, bconv, bias2d) if t is not None]

    def finalize(self):
        n = len(self._jobs)
        arr = (L.PrepJob * n)(*self._jobs)
        L.check(L.lib().stgcn_prep_check(arr, n), "prep_check")
        starts, b = [], 0
        for j in arr:
            starts.append(b)
            b += -(-j.threads // 256)
        starts.append(b)
        self.nblocks = b
        raw = bytes(memoryview(arr).cast("B"))
        self._table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        self._starts = torch.tensor(starts, dtype=torch.int64).to(self.device)
        self.njobs = n
        return self

    def run(self):
        if self._table is None:
            self.finalize()
        L.check(L.lib().stgcn_prep_run(self._table.data_ptr(), self._starts.data_ptr(), self.njobs, self.nblocks,
                                       L.stream()), "prep_run")


def conv_rows(x, w3p, Cin, Cout, cp, kp, T_in, T_out, Kt=1, stride=1, pad=0, trans=False, bias=None, bias_mode=None,
              pro=0, pro_a=None, pro_b=None, pro_stats=None, stats=None, out=None, accumulate=False, tag=None):
    """Implicit-GEMM row conv (stgcn_conv_rows).  x rows: [N, T_in, V, Cin] (any channels-last view).

    Returns ``out`` as a logical (N, Cout, T_out, V) channels-last tensor.
    """
    N, V = x.shape[0], x.shape[3]
    if out is None:
        out = cl_empty(N, Cout, T_out, V, x.dtype, x.device)
    d = L.ConvDesc()
    d.in_, d.out, d.w = x.data_ptr(), out.data_ptr(), w3p.data_ptr()
    fs = getattr(w3p, "frag_stride", None)
    d.w_frag = getattr(w3p, "frag_ptr", None) if fs is not None and fs in (stride, 0) else None
    d.bias = L.ptr(bias)
    d.pro_a, d.pro_b, d.pro_stats = L.ptr(pro_a), L.ptr(pro_b), L.ptr(pro_stats)
    d.stats = L.ptr(stats)
    d.N, d.T_in, d.T_out, d.V, d.Cin, d.Cout, d.Cin_pad, d.Cout_pad = N, T_in, T_out, V, Cin, Cout, kp, cp
    d.Kt, d.stride, d.pad, d.trans, d.pro = Kt, stride, pad, int(trans), pro
    d.bias_mode = (0 if bias is None else 1) if bias_mode is None else bias_mode
    d.accumulate = int(accumulate)
    d.in_ld, d.out_ld = rows_ld(x), rows_ld(out)
    hook = EVENT_HOOK if tag is not None else None
    if hook:  # (tag, phase, algorithmic flops of the launch)
        hook(tag, "start", 2.0 * N * T_out * V * Cout * Cin * Kt)
    h = KTIME_HOOK
    if h:
        fam = ("tcn_dgrad" if trans else "tcn_fwd") if Kt > 1 else "conv1x1"
        ktag = _k_start(h, fam, f"{Cin}->{Cout} s{stride}", 2.0 * N * T_out * V * Cout * Cin * Kt,
                        x.element_size() * N * V * (T_in * Cin + T_out * Cout))
    L.check(L.lib().stgcn_conv_rows(d, L.dtype_code(x.dtype), L.stream()), "conv_rows")
    if h:
        h(ktag, "end", None)
    if hook:
        hook(tag, "end", None)
    return out


def tconv_frame_ok(C, kt, stride, V, dtype) -> bool:
    """Whether a layer's temporal-conv data gradient (C -> C channels) runs on the frame-streaming kernel
    tconv_frame.hip (row-streaming form): bf16, C = 64, Kt = 9, stride 1, 16 < V <= 25 (46 vs 65 us for conv_persist,
    DESIGN 4.14)."""
    return dtype == torch.bfloat16 and C == 64 and kt == 9 and stride == 1 and 16 < V <= 25


def tconv_frame_row_blocks(N: int, T: int) -> int:
    return L.lib().stgcn_tconv_frame_row_blocks(N, T)


def tconv_frame(x, w3p, cp, kp, trans=False, bias=None, pro_a=None, pro_b=None, stats=None, tag=None):
    """The 64-channel Kt = 9 stride-1 temporal conv (forward: BN1 scale / shift + ReLU prologue when pro_a is given,
    bias, BN partials; trans: the data gradient) on the frame-streaming kernel (stgcn_tconv_frame); w3p a
    pack_weight result carrying its stride-1 fragment image.  Returns the (N, 64, T, V) channels-last output."""
    N, C, T, V = x.shape
    if getattr(w3p, "frag_stride", None) != 1:
        raise RuntimeError("stgcn_amd: tconv_frame needs the stride-1 fragment image of the weight")
    out = cl_empty(N, C, T, V, x.dtype, x.device)
    d = L.ConvDesc()
    d.in_, d.out, d.w, d.w_frag = x.data_ptr(), out.data_ptr(), w3p.data_ptr(), w3p.frag_ptr
    d.bias, d.pro_a, d.pro_b, d.stats = L.ptr(bias), L.ptr(pro_a), L.ptr(pro_b), L.ptr(stats)
    d.N, d.T_in, d.T_out, d.V, d.Cin, d.Cout, d.Cin_pad, d.Cout_pad = N, T, T, V, C, C, kp, cp
    d.Kt, d.stride, d.pad, d.trans, d.pro = 9, 1, 4, int(trans), 1 if pro_a is not None else 0
    d.bias_mode, d.accumulate = 0 if bias is None else 1, 0
    d.in_ld, d.out_ld = rows_ld(x), rows_ld(out)
    hook = EVENT_HOOK if tag is not None else None
    flop = 2.0 * N * T * V * C * C * 9
    if hook:
        hook(tag, "start", flop)
    h = KTIME_HOOK
    if h:
        ktag = _k_start(h, "tconv_frame_dgrad" if trans else "tconv_frame_fwd", f"{C}->{C} s1", flop,
                        x.element_size() * N * V * T * 2 * C)
    L.check(L.lib().stgcn_tconv_frame(d, L.stream()), "tconv_frame")
    if h:
        h(ktag, "end", None)
    if hook:
        hook(tag, "end", None)
    return out


def conv_wgrad(x, dy, Cin, Cout, T_in, T_out, Kt=1, stride=1, pad=0, pro=0, pro_a=None, pro_b=None, pro_stats=None,
               dw=None):
    """dw[Kt][Cout][Cin] (fp32) += weight gradient (stgcn_conv_wgrad)."""
    N, V = x.shape[0], x.shape[3]
    if dw is None:
        dw = torch.zeros((Kt, Cout, Cin), dtype=torch.float32, device=x.device)
    d = L.WgradDesc()
    d.in_, d.dy, d.dw = x.data_ptr(), dy.data_ptr(), dw.data_ptr()
    d.pro_a, d.pro_b, d.pro_stats = L.ptr(pro_a), L.ptr(pro_b), L.ptr(pro_stats)
    d.N, d.T_in, d.T_out, d.V, d.Cin, d.Cout, d.Kt, d.stride, d.pad, d.pro = \
        N, T_in, T_out, V, Cin, Cout, Kt, stride, pad, pro
    d.in_ld, d.dy_ld = rows_ld(x), rows_ld(dy)
    code = L.dtype_code(x.dtype)
    nbytes = L.lib().stgcn_conv_wgrad_workspace(d, code)
    if nbytes > 0:  # per-block fp32 partials of the deterministic frame-tiled path
        work = torch.empty(nbytes // 4, dtype=torch.float32, device=x.device)
        d.work, d.work_bytes = work.data_ptr(), nbytes
    L.check(L.lib().stgcn_conv_wgrad(d, code, L.stream()), "conv_wgrad")
    return dw


def conv_wgrad_w(x, dy, Cin, Cout, T_in, T_out, Kt=1, stride=1, pad=0, pro=0, pro_a=None, pro_b=None, pro_stats=None):
    """The weight gradient as a FRESH fp32 tensor in nn.Conv2d weight order (Cout, Cin, Kt): the workspace paths
    write it directly (out_mode 1: no zero fill, no permute copy); the others accumulate into zeros and permute."""
    N, V = x.shape[0], x.shape[3]
    d = L.WgradDesc()
    d.in_, d.dy = x.data_ptr(), dy.data_ptr()
    d.pro_a, d.pro_b, d.pro_stats = L.ptr(pro_a), L.ptr(pro_b), L.ptr(pro_stats)
    d.N, d.T_in, d.T_out, d.V, d.Cin, d.Cout, d.Kt, d.stride, d.pad, d.pro = \
        N, T_in, T_out, V, Cin, Cout, Kt, stride, pad, pro
    d.in_ld, d.dy_ld = rows_ld(x), rows_ld(dy)
    code = L.dtype_code(x.dtype)
    nbytes = L.lib().stgcn_conv_wgrad_workspace(d, code)
    if nbytes <= 0:
        return conv_wgrad(x, dy, Cin, Cout, T_in, T_out, Kt, stride, pad, pro, pro_a, pro_b,
                          pro_stats).permute(1, 2, 0).contiguous()
    work = torch.empty(nbytes // 4, dtype=torch.float32, device=x.device)
    d.work, d.work_bytes = work.data_ptr(), nbytes
    dw = torch.empty((Cout, Cin, Kt), dtype=torch.float32, device=x.device)
    d.dw, d.out_mode = dw.data_ptr(), 1
    h = KTIME_HOOK
    if h:
        ktag = _k_start(h, "tcn_wgrad" if Kt > 1 else "wgrad1x1", f"{Cin}->{Cout} s{stride}",
                        2.0 * N * T_out * V * Cout * Cin * Kt, x.element_size() * N * V * (T_in * Cin + T_out * Cout))
    L.check(L.lib().stgcn_conv_wgrad(d, code, L.stream()), "conv_wgrad")
    if h:
        h(ktag, "end", None)
    return dw


def _amix_desc(x, out, A, N, T, V, P, Cin, accumulate=False, x_ld=None, out_ld=None):
    A = _dense(A)
    d = L.AmixDesc()
    d._keep = A  # a dense copy must outlive the descriptor's launch
    d.x, d.out, d.A = x.data_ptr(), L.ptr(out), A.data_ptr()
    d.N, d.T, d.V, d.P, d.Cin = N, T, V, P, Cin
    d.per_sample = int(A.dim() == 4)
    d.accumulate = int(accumulate)
    d.x_ld = x_ld if x_ld is not None else rows_ld(x)
    d.out_ld = out_ld if out_ld is not None else (rows_ld(out) if out is not None else 0)
    return d


def amix_fwd(x, A):
    """XA (N, P*Cin, T, V) channels-last = A-mix of x (stgcn_amix_fwd)."""
    N, Cin, T, V = x.shape
    P = A.shape[-3]
    out = cl_empty(N, P * Cin, T, V, x.dtype, x.device)
    d = _amix_desc(x, out, A, N, T, V, P, Cin)
    L.check(L.lib().stgcn_amix_fwd(d, L.dtype_code(x.dtype), L.stream()), "amix_fwd")
    return out


def amix_trans(dw, A, Cin, out, accumulate):
    """out (N,Cin,T,V) (+)= A^T-mix of DW (N, P*Cin, T, V) (stgcn_amix_trans)."""
    N, _, T, V = dw.shape
    P = A.shape[-3]
    d = _amix_desc(dw, out, A, N, T, V, P, Cin, accumulate)
    L.check(L.lib().stgcn_amix_trans(d, L.dtype_code(dw.dtype), L.stream()), "amix_trans")
    return out


def zeros_arena(device, *shapes):
    """Zeroed fp32 tensors of the given shapes carved from ONE allocation (one fill launch instead of one
    per buffer); every view starts 256-B aligned."""
    sizes = [int(torch.Size(sh).numel()) for sh in shapes]
    offs, tot = [], 0
    for n in sizes:
        offs.append(tot)
        tot += -(-n // 64) * 64
    buf = torch.zeros(max(tot, 1), dtype=torch.float32, device=device)
    return [buf[o:o + n].view(sh) for o, n, sh in zip(offs, sizes, shapes)]


def _workspace(nbytes, device):
    """fp32 scratch of at least nbytes (>= 1 element so data_ptr is valid)."""
    return torch.empty(max(1, (nbytes + 3) // 4), dtype=torch.float32, device=device)


def amix_dA(x, dw, A):
    """dA (fp32, shape of A) = sum x (x) DW (stgcn_amix_dA)."""
    N, Cin, T, V = x.shape
    P = A.shape[-3]
    dA = torch.zeros(A.shape, dtype=torch.float32, device=x.device)
    d = _amix_desc(x, None, A, N, T, V, P, Cin)
    # per-block partials + fixed-order reduction: bit-reproducible (no atomics)
    work = _workspace(L.lib().stgcn_amix_dA_workspace(d), x.device)
    L.check(L.lib().stgcn_amix_dA(d, dw.data_ptr(), dA.data_ptr(), work.data_ptr(), L.dtype_code(x.dtype),
                                  L.stream()), "amix_dA")
    return dA


def gcn_bias_bwd(A, b, S, dA, C):
    """Shared A: dA += bias-through-A term (in place), returns db [P*C] (stgcn_gcn_bias_bwd)."""
    A = _dense(A)
    P, V = A.shape[0], A.shape[-1]
    db = torch.empty(P * C, dtype=torch.float32, device=A.device)
    L.check(L.lib().stgcn_gcn_bias_bwd(A.data_ptr(), b.data_ptr(), S.data_ptr(), P, V, C, dA.data_ptr(),
                                       db.data_ptr(), L.stream()), "gcn_bias_bwd")
    return db


def gcn_bias(A, b, N, C):
    """bias2d [V, C] (shared A) or [N, V, C] (per-sample A) = sum_p b_p * colsum(A_p)."""
    A = _dense(A)
    P, V = A.shape[-3], A.shape[-1]
    per = A.dim() == 4
    out = torch.empty(((N,) if per else ()) + (V, C), dtype=torch.float32, device=A.device)
    L.check(L.lib().stgcn_gcn_bias(A.data_ptr(), b.data_ptr(), out.data_ptr(), N, P, V, C, int(per), L.stream()),
            "gcn_bias")
    return out


# ------------------------------------------------------------------------------ graph conv (gather GEMM)
class GraphSupport:
    """Support lists of a batch-shared adjacency A [P][V][V] for stgcn_gconv: S(w) = {v : A[:, v, w] != 0}
    (forward) and R(v) = {w : A[:, v, w] != 0} (data grad), padded to J = max degree, on the device."""

    def __init__(self, A):
        import numpy as np
        a = (A.detach().abs().sum(0) > 0).cpu().numpy()  # [v][w]
        V = a.shape[0]
        self.V = V
        S = [np.nonzero(a[:, w])[0] for w in range(V)]
        R = [np.nonzero(a[v, :])[0] for v in range(V)]
        self.J = max(1, max(len(s) for s in S), max(len(r) for r in R))
        self.nnz = int(a.sum())
        self.mask = torch.as_tensor(a, device=A.device)

        def pack(lists):
            nb = np.full((V, self.J), 0, dtype=np.int32)
            dg = np.zeros(V, dtype=np.int32)
            for i, l in enumerate(lists):
                nb[i, :len(l)] = l
                dg[i] = len(l)
            return torch.as_tensor(nb, device=A.device), torch.as_tensor(dg, device=A.device)

        self.nbr, self.deg = pack(S)
        self.rnbr, self.rdeg = pack(R)

    def dense(self, P):
        """A-first (amix) is cheaper when the support is denser than P entries per output joint."""
        return self.nnz > P * self.V


def gconv_weights(A, W, sup, Cout, Cin, trans, dtype, bias=None, plan=None, M=None):
    """Effective weights [V][J][R_pad][C_pad]: trans 0 -> (Cout, Cin) from S lists, 1 -> (Cin, Cout) from R lists.

    ``bias`` (forward only: the conv bias, fp32 [P*Cout]): the same launch also pushes it through A
    (stgcn_gconv_weights_bias), and the call returns (weights, bias2d [V][Cout]) — gcn_bias's result.
    ``plan``: record the job in a PrepPlan instead of launching; the coefficients are then A * M (``M`` the
    layer's edge importance, or None), formed inside the batched launch."""
    A = _dense(A)
    P, V = A.shape[0], A.shape[-1]
    R, C = (Cin, Cout) if trans else (Cout, Cin)
    rp = -(-R // col_tile(R)) * col_tile(R)
    cpad = -(-C // 32) * 32
    out = torch.empty((V, sup.J, rp, cpad), dtype=dtype, device=A.device)
    if plan is not None:
        nbr, deg = (sup.rnbr, sup.rdeg) if trans else (sup.nbr, sup.deg)
        plan.add(kind=2, dtype=L.dtype_code(dtype), src=W, dst=out, Co=Cout, Ci=Cin, trans=int(trans), A=A,
                 M=None if M is None else _dense(M), nbr=nbr, deg=deg, P=P, V=V, J=sup.J, R_pad=rp, C_pad=cpad)
        # the bias through A as its own job (kind 3, the same per-output sum): a kind-2 job carrying it had every
        # one of its blocks compute the column sums of A * M before its first weight load
        return (out, gcn_bias_plan(A, bias, Cout, plan, M)) if bias is not None else out
    if bias is not None:
        assert not trans
        b2 = torch.empty((V, Cout), dtype=torch.float32, device=A.device)
        L.check(L.lib().stgcn_gconv_weights_bias(A.data_ptr(), W.data_ptr(), bias.data_ptr(), sup.nbr.data_ptr(),
                                                 sup.deg.data_ptr(), P, V, sup.J, Cout, Cin, out.data_ptr(), rp, cpad,
                                                 b2.data_ptr(), L.dtype_code(dtype), L.stream()), "gconv_weights_bias")
        return out, b2
    nbr, deg = (sup.rnbr, sup.rdeg) if trans else (sup.nbr, sup.deg)
    L.check(L.lib().stgcn_gconv_weights(A.data_ptr(), W.data_ptr(), nbr.data_ptr(), deg.data_ptr(), P, V, sup.J,
                                        Cout, Cin, int(trans), out.data_ptr(), rp, cpad, L.dtype_code(dtype),
                                        L.stream()), "gconv_weights")
    return out


def gconv_row_blocks(NT: int, V: int) -> int:
    return L.lib().stgcn_gconv_row_blocks(NT, V)


def pack_frag1(w2: torch.Tensor, dtype) -> tuple:
    """[Cout][K] fp32 1x1 weight -> its MFMA-fragment image (stgcn_pack_weight_frag, Kt = 1):
    (image, Cout_pad, K_pad)."""
    Co, Ci = w2.shape
    cp = -(-Co // col_tile(Co)) * col_tile(Co)
    kp = -(-Ci // 32) * 32
    if w2.dtype != torch.float32:
        w2 = w2.float()
    buf = torch.empty(2 * cp * kp, dtype=dtype, device=w2.device)
    s1, s2 = w2.stride()
    L.check(L.lib().stgcn_pack_weight_frag(w2.data_ptr(), 0, s1, s2, 1, Co, Ci, buf.data_ptr(), buf[cp * kp:].data_ptr(),
                                           cp, kp, L.dtype_code(dtype), L.stream()), "pack_weight_frag")
    return buf[cp * kp:], cp, kp


_PERM16 = {}


def pack_gcn_weight(w2: torch.Tensor, dtype) -> tuple:
    """[Cout][P*Cin] fp32 W' -> the graph-conv weight image of stgcn_layer_fused_fwd (wg_frag): the Kt = 1 fragment
    image of W' with the columns of every 16-wide group in the order of the joint-mix accumulators' rows
    (include/stgcn_amd.h): (image, Cout_pad, K_pad)."""
    K = w2.shape[1]
    key = (K, w2.device)
    perm = _PERM16.get(key)
    if perm is None:
        h = torch.arange(16) // 8
        j = torch.arange(16) % 8
        within = 8 * (j // 4) + 4 * h + j % 4
        perm = (torch.arange(K) // 16 * 16 + within.repeat(K // 16)).to(w2.device)
        _PERM16[key] = perm
    return pack_frag1(w2.float().index_select(1, perm), dtype)


def gcn_bias_plan(A, b, Cout, plan, M=None):
    """bias2d [V][Cout] = sum_p b_p colsum_p(A * M) recorded as a PrepPlan job (kind 3)."""
    A = _dense(A)
    P, V = A.shape[0], A.shape[-1]
    b2 = torch.empty((V, Cout), dtype=torch.float32, device=A.device)
    bc = b.detach()
    plan.add(kind=3, dtype=1, src=bc.view(1, -1), dst=b2, Co=Cout, Ci=1, A=A, M=None if M is None else _dense(M), P=P, V=V,
             bconv=bc, bias2d=b2)
    return b2


def layer_fused_ok(sup, P, Cin, Cout, V, kt, stride, dtype) -> bool:
    """Whether a LayerNorm layer's forward can run as the one-kernel layer (layer_fused.hip): bf16, 64 -> 64
    channels, stride 1, Kt = 9, a batch-shared graph, 16 < V <= 25.  A shape check only: each caller tests its
    own routing switch (fused_inference, fused_ln_train)."""
    return (dtype == torch.bfloat16 and sup is not None and P <= 3 and 16 < V <= 25
            and Cin == 64 and Cout == 64 and kt == 9 and stride == 1)


def layer_fused(x, A, wimg, gbias, wt_packed, tbias, ln, tag=None, residual=False, train=False):
    """stgcn_layer_fused_fwd: the whole LayerNorm layer y = relu(LN2(tcn(relu(LN1(gcn(x))))) + residual * x) in one
    kernel; ln = (g1, b1, g2, b2) LayerNorm parameters as [V][64] fp32.  ``train``: also the backward's inputs —
    returns (y, g, u, ls1, ls2, h): g / u the graph-conv / temporal-conv outputs (bias included) as rows, ls1 / ls2
    their per-frame (mean, rstd) [N*T][2] (ln_stats's layout), h = relu(LN1(g))."""
    N, C, T, V = x.shape
    if getattr(wt_packed, "frag_stride", None) != 1:
        raise RuntimeError("stgcn_amd: layer_fused needs the stride-1 fragment image of the temporal weight")
    z = cl_empty(N, C, T, V, x.dtype, x.device)
    A = _dense(A)
    d = L.LayerFusedDesc()
    d.x, d.z, d.wg_frag, d.A = x.data_ptr(), z.data_ptr(), wimg.data_ptr(), A.data_ptr()
    d.gbias, d.wt_frag, d.tbias = L.ptr(gbias), wt_packed.frag_ptr, L.ptr(tbias)
    d.N, d.T, d.V, d.P, d.x_ld, d.z_ld = N, T, V, A.shape[0], rows_ld(x), rows_ld(z)
    ln = [_f32c(t) for t in ln]
    if any(t.numel() != V * C for t in ln):
        raise RuntimeError("stgcn_amd: layer_fused LayerNorm parameters must be [V][64]")
    d.ln1_g, d.ln1_b, d.ln2_g, d.ln2_b = (t.data_ptr() for t in ln)
    d.residual = int(bool(residual))
    d._keep = ln
    if train:
        g = cl_empty(N, C, T, V, x.dtype, x.device)
        u = cl_empty(N, C, T, V, x.dtype, x.device)
        st = torch.empty((2, N * T, 2), dtype=torch.float32, device=x.device)
        d.g_out, d.u_out, d.st1_out, d.st2_out = g.data_ptr(), u.data_ptr(), st[0].data_ptr(), st[1].data_ptr()
        d.g_ld, d.u_ld = rows_ld(g), rows_ld(u)
        hh = cl_empty(N, C, T, V, x.dtype, x.device)
        d.h_out, d.h_ld = hh.data_ptr(), rows_ld(hh)
    hook = EVENT_HOOK if tag is not None else None
    if hook:
        hook(tag, "start", None)
    L.check(L.lib().stgcn_layer_fused_fwd(d, L.stream()), "layer_fused")
    if hook:
        hook(tag, "end", None)
    if train:
        return z, g, u, st[0], st[1], hh
    return z


def gconv(x, wpk, sup, Cin, Cout, trans=False, bias=None, stats=None, out=None, accumulate=False, tag=None,
          res=None):
    """out rows (N, Cout, T, V) (+)= joint-gathered GEMM of x rows with packed effective weights.
    ``res`` = (rows, sign bits): out = GEMM + rows * mask (bf16; the identity residual's masked gradient)."""
    N, _, T, V = x.shape
    if out is None:
        out = cl_empty(N, Cout, T, V, x.dtype, x.device)
    nbr, deg = (sup.rnbr, sup.rdeg) if trans else (sup.nbr, sup.deg)
    d = L.GconvDesc()
    d.in_, d.out, d.w = x.data_ptr(), out.data_ptr(), wpk.data_ptr()
    d.nbr, d.deg, d.bias, d.stats = nbr.data_ptr(), deg.data_ptr(), L.ptr(bias), L.ptr(stats)
    d.NT, d.V, d.J, d.Cin, d.Cout = N * T, V, sup.J, Cin, Cout
    d.Cin_pad, d.Cout_pad = wpk.shape[3], wpk.shape[2]
    d.in_ld, d.out_ld, d.accumulate = rows_ld(x), rows_ld(out), int(accumulate)
    if res is not None:
        rr, rbits = res
        if accumulate or rbits.dtype != torch.uint8:
            raise RuntimeError("stgcn_amd: gconv's masked residual needs accumulate=False and uint8 sign bits")
        d.res, d.res_bits, d.res_ld = rr.data_ptr(), rbits.data_ptr(), rows_ld(rr)
    h = KTIME_HOOK
    if h:
        ktag = _k_start(h, "gconv_dgrad" if trans else "gconv_fwd", f"{Cin}->{Cout}" if not trans else f"{Cout}->{Cin}",
                        2.0 * N * T * sup.nnz * Cin * Cout,
                        x.element_size() * N * T * V * (Cin + Cout * (2 if accumulate else 1)))
    L.check(L.lib().stgcn_gconv(d, L.dtype_code(x.dtype), L.stream()), "gconv")
    if h:
        h(ktag, "end", None)
    return out


def gconv_wgrad_rowsum_ok(sup, Cin, Cout, dtype) -> bool:
    """Whether gconv_wgrad can also return the per-joint row sums of dy (joint-grouped kernel only)."""
    return dtype == torch.bfloat16 and Cin % 64 == 0 and Cout % 64 == 0 and sup.J <= 5


def gconv_wgrad(x, dy, sup, Cin, Cout, rowsum=None):
    """dWeff [V][J][Cout][Cin] fp32 = sum_i dy[(i,w)] x[(i, S(w)_j)]^T; with ``rowsum`` ([V][Cout] fp32,
    overwritten) also the per-joint row sums of dy (gconv_wgrad_rowsum_ok shapes)."""
    N, _, T, V = x.shape
    dweff = torch.empty((V, sup.J, Cout, Cin), dtype=torch.float32, device=x.device)
    d = L.GconvWgradDesc()
    d.rowsum = L.ptr(rowsum)
    d.x, d.dy, d.nbr, d.deg, d.dweff = x.data_ptr(), dy.data_ptr(), sup.nbr.data_ptr(), sup.deg.data_ptr(), \
        dweff.data_ptr()
    d.NT, d.V, d.J, d.Cin, d.Cout, d.x_ld, d.dy_ld = N * T, V, sup.J, Cin, Cout, rows_ld(x), rows_ld(dy)
    code = L.dtype_code(x.dtype)
    nbytes = L.lib().stgcn_gconv_wgrad_workspace(d, code)
    if nbytes > 0:
        work = torch.empty(nbytes // 4, dtype=torch.float32, device=x.device)
        d.work, d.work_bytes = work.data_ptr(), nbytes
    h = KTIME_HOOK
    if h:
        ktag = _k_start(h, "gconv_wgrad", f"{Cin}->{Cout}", 2.0 * N * T * sup.nnz * Cin * Cout,
                        x.element_size() * N * T * V * (Cin + Cout))
    hook = EVENT_HOOK
    if hook and gconv_wgrad3_shape(sup, Cin, Cout, x.dtype):
        # bench.py's roofline: the accumulation kernel (gconv_wgrad3) bracketed alone, then its slab reduction
        d.phase = 1
        hook("gconv_wgrad3", "start", {"flop": 2.0 * N * T * sup.nnz * Cin * Cout,
                                       "bytes": x.element_size() * N * T * V * (Cin + Cout), "shape": f"{Cin}->{Cout}"})
        L.check(L.lib().stgcn_gconv_wgrad(d, code, L.stream()), "gconv_wgrad")
        hook("gconv_wgrad3", "end", None)
        d.phase = 2
    L.check(L.lib().stgcn_gconv_wgrad(d, code, L.stream()), "gconv_wgrad")
    if h:
        h(ktag, "end", None)
    return dweff


def gconv_wgrad3_shape(sup, Cin, Cout, dtype) -> bool:
    """Whether stgcn_gconv_wgrad runs the DMA-ring kernel gconv_wgrad3 for this shape (gconv.hip w2_cob / w3_ok:
    bf16, channels % 64, <= 5 neighbours, not 64 -> 128)."""
    return dtype == torch.bfloat16 and Cin % 64 == 0 and Cout % 64 == 0 and sup.J <= 5 and not (Cin == 64 and Cout == 128)


def gconv_finish(dweff, A, W, sup, Cout, Cin, dW=None, dA=None):
    """(dW [P*Cout][Cin], dA [P][V][V]) fp32 (+)= from dWeff (stgcn_gconv_wgrad_finish); zeroed if not given."""
    A = _dense(A)
    P, V = A.shape[0], A.shape[-1]
    if dW is None:
        dW = torch.zeros((P * Cout, Cin), dtype=torch.float32, device=A.device)
    if dA is None:
        dA = torch.zeros((P, V, V), dtype=torch.float32, device=A.device)
    work = _workspace(L.lib().stgcn_gconv_wgrad_finish_workspace(P, V, sup.J, Cout, Cin), A.device)
    L.check(L.lib().stgcn_gconv_wgrad_finish(dweff.data_ptr(), A.data_ptr(), W.data_ptr(), sup.nbr.data_ptr(),
                                             sup.deg.data_ptr(), P, V, sup.J, Cout, Cin, dW.data_ptr(), dA.data_ptr(),
                                             work.data_ptr(), L.stream()), "gconv_finish")
    return dW, dA


def gconv_finish_bias(dweff, A, W, sup, Cout, Cin, bconv, S):
    """(dW [P*Cout][Cin], dA [P][V][V], db [P*Cout]) fp32, all overwritten (stgcn_gconv_wgrad_finish_bias): the
    graph-conv weight / adjacency gradient from dWeff with the conv bias pushed through A (S = per-joint row sums
    of dy [V][Cout]) in two launches; fresh outputs, no zero fill."""
    A = _dense(A)
    P, V = A.shape[0], A.shape[-1]
    dev = A.device
    out = torch.empty(P * Cout * Cin + P * V * V + P * Cout, dtype=torch.float32, device=dev)
    dW = out[:P * Cout * Cin].view(P * Cout, Cin)
    dA = out[P * Cout * Cin:P * Cout * Cin + P * V * V].view(P, V, V)
    db = out[P * Cout * Cin + P * V * V:]
    work = _workspace(L.lib().stgcn_gconv_wgrad_finish_workspace(P, V, sup.J, Cout, Cin), dev)
    h = KTIME_HOOK
    if h:
        ktag = _k_start(h, "gconv_wgrad_finish", f"{Cin}->{Cout}", None, 4 * dweff.numel())
    L.check(L.lib().stgcn_gconv_wgrad_finish_bias(dweff.data_ptr(), A.data_ptr(), W.data_ptr(), sup.nbr.data_ptr(),
                                                  sup.deg.data_ptr(), P, V, sup.J, Cout, Cin, bconv.data_ptr(),
                                                  S.data_ptr(), dW.data_ptr(), dA.data_ptr(), db.data_ptr(),
                                                  work.data_ptr(), L.stream()), "gconv_finish_bias")
    if h:
        h(ktag, "end", None)
    return dW, dA, db


def gconv_finish_bias_ok(A, sup) -> bool:
    return A.dim() == 3 and A.shape[0] <= 4 and A.shape[-1] <= 32 and A.shape[-1] * sup.J <= 256


def bn_stat_blocks(M: int) -> int:
    return L.lib().stgcn_bn_stat_blocks(M)


def bn_stats_partial(x, M, C, ld=None):
    nb = bn_stat_blocks(M)
    part = torch.empty((nb, C, 4), dtype=torch.float32, device=x.device)
    L.check(L.lib().stgcn_bn_stats_partial(x.data_ptr(), ld or rows_ld(x), M, C, part.data_ptr(),
                                           L.dtype_code(x.dtype), L.stream()), "bn_stats_partial")
    return part, nb, C


def bn_finalize(part, nb, ld_part, C, gamma, beta, eps=1e-5):
    buf = torch.empty(4 * C, dtype=torch.float32, device=part.device)  # (mean, rstd) pairs | scale | shift
    mr, sc, sh = buf[:2 * C].view(C, 2), buf[2 * C:3 * C], buf[3 * C:]
    L.check(L.lib().stgcn_bn_finalize(part.data_ptr(), nb, ld_part, C, L.ptr(gamma), L.ptr(beta), eps, mr.data_ptr(),
                                      sc.data_ptr(), sh.data_ptr(), L.stream()), "bn_finalize")
    return mr, sc, sh


def bn_merge(part, nb, ld_part, C):
    """[C][4] float32: the nb (count, mean, M2) partials of each channel merged into one entry (stgcn_bn_merge) —
    a rank's SyncBatchNorm contribution; the gathered [ranks][C][4] entries go through bn_finalize(nb = ranks)."""
    out = torch.empty((C, 4), dtype=torch.float32, device=part.device)
    L.check(L.lib().stgcn_bn_merge(part.data_ptr(), nb, ld_part, C, out.data_ptr(), L.stream()), "bn_merge")
    return out


def bn_apply(u, sc, sh, M, C, res_mode=0, r=None, rsc=None, rsh=None, relu=True, out=None, ldu=None, ldy=None,
             bits=None):
    """y = act(u*sc + sh + res) (stgcn_bn_apply).  ``bits`` (uint8 [M][C/8], bf16 and C % 8 == 0 only): also the
    output's sign bits (stgcn_bn_apply_bits), the backward's ReLU mask at 1/16 of y's bytes (bn_bwd_fused mask 3)."""
    if out is None:
        out = torch.empty_like(u)
    h = KTIME_HOOK
    if h:
        ktag = _k_start(h, "bn_apply", f"C{C}", None, u.element_size() * M * C * (3 if r is not None else 2))
    args = (u.data_ptr(), ldu or rows_ld(u), sc.data_ptr(), sh.data_ptr(), res_mode, L.ptr(r),
            rows_ld(r) if r is not None else 0, L.ptr(rsc), L.ptr(rsh), int(relu), out.data_ptr(),
            ldy or rows_ld(out), M, C)
    if bits is not None:
        if u.dtype != torch.bfloat16 or C % 8 or bits.dtype != torch.uint8 or bits.numel() < M * (C // 8):
            raise RuntimeError("stgcn_amd: bn_apply bits need bf16 rows, C % 8 == 0 and a uint8 [M][C/8] buffer")
        L.check(L.lib().stgcn_bn_apply_bits(*args, bits.data_ptr(), L.stream()), "bn_apply_bits")
    else:
        L.check(L.lib().stgcn_bn_apply(*args, L.dtype_code(u.dtype), L.stream()), "bn_apply")
    if h:
        h(ktag, "end", None)
    return out


def bn_bwd_reduce(dy, M, C, mask=0, mref=None, msc=None, msh=None, x=None, mean_rstd=None, lddy=None):
    nb = bn_stat_blocks(M)
    part = torch.empty((nb, C, 2), dtype=torch.float32, device=dy.device)
    sums = torch.empty((C, 2), dtype=torch.float32, device=dy.device)
    L.check(L.lib().stgcn_bn_bwd_reduce(dy.data_ptr(), lddy or rows_ld(dy), mask, L.ptr(mref),
                                        rows_ld(mref) if mref is not None else 0, L.ptr(msc), L.ptr(msh), L.ptr(x),
                                        rows_ld(x) if x is not None else 0, L.ptr(mean_rstd), M, C, part.data_ptr(),
                                        sums.data_ptr(), L.dtype_code(dy.dtype), L.stream()), "bn_bwd_reduce")
    return sums


def bn_bwd_apply(dy, M, C, out, mask=0, mref=None, msc=None, msh=None, x=None, mean_rstd=None, gamma=None,
                 sums=None, accumulate=False, lddy=None):
    L.check(L.lib().stgcn_bn_bwd_apply(dy.data_ptr(), lddy or rows_ld(dy), mask, L.ptr(mref),
                                       rows_ld(mref) if mref is not None else 0, L.ptr(msc), L.ptr(msh), L.ptr(x),
                                       rows_ld(x) if x is not None else 0, L.ptr(mean_rstd), L.ptr(gamma),
                                       L.ptr(sums), M, C, out.data_ptr(), rows_ld(out), int(accumulate),
                                       L.dtype_code(dy.dtype), L.stream()), "bn_bwd_apply")
    return out


def bn_fused_ok(C: int, dtype) -> bool:
    vec = 8 if dtype == torch.bfloat16 else 4
    return C % vec == 0 and C // vec <= 256


def bn_bwd_fused(dy, M, C, mask=0, mref=None, msc=None, msh=None, x1=None, mr1=None, g1=None, out1=None,
                 x2=None, mr2=None, g2=None, out2=None, acc2=False, bias_sums=False, sync=None):
    # mask 3: mref = the uint8 [M][C/8] sign bits of the forward's output (bn_apply(bits=...))
    """Fused BN backward (stgcn_bn_bwd_fused_*).  Returns (sums [3, C] = (sum dz, sum dz*xhat1, sum dz*xhat2),
    osum [3, C] = (sum out1, sum out2, -) or None), contiguous rows.  out1 / out2 are written in place.
    ``sync`` (syncbn.BnSync): SyncBatchNorm — the apply pass uses the sums of every rank (exchanged between the
    two passes); the returned sums stay this rank's own (the parameter gradients, which DDP then averages)."""
    code = L.dtype_code(dy.dtype)
    dev = dy.device
    work = torch.empty(L.lib().stgcn_bn_bwd_fused_workspace(M, C, code), dtype=torch.float32, device=dev)
    sums = torch.empty(7 * C, dtype=torch.float32, device=dev)
    osum = torch.empty(7 * C, dtype=torch.float32, device=dev) if bias_sums else None
    d = L.BnBwdDesc()
    d.dy, d.mref, d.x1, d.x2 = dy.data_ptr(), L.ptr(mref), L.ptr(x1), L.ptr(x2)
    d.msc, d.msh, d.mean_rstd1, d.mean_rstd2 = L.ptr(msc), L.ptr(msh), L.ptr(mr1), L.ptr(mr2)
    d.gamma1, d.gamma2, d.sums = L.ptr(g1), L.ptr(g2), sums.data_ptr()
    d.out1, d.out2, d.osum, d.work = L.ptr(out1), L.ptr(out2), L.ptr(osum), work.data_ptr()
    d.M, d.C, d.mask = M, C, mask
    d.lddy = rows_ld(dy)
    d.ldm = (C // 8 if mask == 3 else rows_ld(mref)) if mref is not None else 0
    d.ldx1 = rows_ld(x1) if x1 is not None else 0
    d.ldx2 = rows_ld(x2) if x2 is not None else 0
    d.ldo1 = rows_ld(out1) if out1 is not None else 0
    d.ldo2 = rows_ld(out2) if out2 is not None else 0
    d.acc2 = int(acc2)
    h = KTIME_HOOK
    es = dy.element_size()
    n_in = sum(t is not None for t in (dy, mref, x1, x2))
    if h:
        ktag = _k_start(h, "bn_bwd_reduce", f"C{C}", None, es * M * C * n_in)
    L.check(L.lib().stgcn_bn_bwd_fused_reduce(d, code, L.stream()), "bn_bwd_fused_reduce")
    if h:
        h(ktag, "end", None)
    if sync is not None and out1 is not None:
        # the reduce pass wrote the per-channel sums twice: float4 rows [C] (what apply reads) and planar [3][C]
        # (returned); only the rows are exchanged
        sync.all_reduce_sums(sums[:4 * C].view(C, 4), M, count_lane=True)
    if out1 is not None:
        if h:
            n_out = 1 + (out2 is not None) * (2 if acc2 else 1)
            ktag = _k_start(h, "bn_bwd_apply", f"C{C}", None, es * M * C * (n_in + n_out))
        L.check(L.lib().stgcn_bn_bwd_fused_apply(d, code, L.stream()), "bn_bwd_fused_apply")
        if h:
            h(ktag, "end", None)
    return sums[4 * C:].view(3, C), (osum[4 * C:].view(3, C) if osum is not None else None)


def rowgroup_sum(x, M, C, G, per_sample=False, out=None):
    """[G][C] (or [N][G][C] per sample) sums of rows grouped by m % G (+= into a zeroed ``out`` if given)."""
    N = x.shape[0]
    S = out if out is not None else \
        torch.zeros(((N,) if per_sample else ()) + (G, C), dtype=torch.float32, device=x.device)
    period = M // N if per_sample else 0
    work = torch.empty(L.lib().stgcn_rowgroup_sum_workspace(M, C, G, period), dtype=torch.float32, device=x.device)
    L.check(L.lib().stgcn_rowgroup_sum(x.data_ptr(), rows_ld(x), M, C, G, period, S.data_ptr(), work.data_ptr(),
                                       L.dtype_code(x.dtype), L.stream()), "rowgroup_sum")
    return S


def cast_colsum(x, M, C):
    """(bf16 channels-last copy of the fp32 rows x, fp32 column sums [C]) from one pass (stgcn_cast_colsum)."""
    out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    cs = torch.empty(C, dtype=torch.float32, device=x.device)
    work = torch.empty(max(L.lib().stgcn_cast_colsum_workspace(M, C), 1), dtype=torch.float32, device=x.device)
    L.check(L.lib().stgcn_cast_colsum(x.data_ptr(), rows_ld(x), M, C, out.data_ptr(), rows_ld(out), cs.data_ptr(),
                                      work.data_ptr(), L.stream()), "cast_colsum")
    return out, cs


# ------------------------------------------------------------------------------------ LayerNorm
def ln_stats(x, frames, V, C, eps=1e-5):
    st = torch.empty((frames, 2), dtype=torch.float32, device=x.device)
    L.check(L.lib().stgcn_ln_stats(x.data_ptr(), rows_ld(x), frames, V, C, eps, st.data_ptr(),
                                   L.dtype_code(x.dtype), L.stream()), "ln_stats")
    return st


def ln_apply(u, st, g, b, M, V, C, res_mode=0, r=None, rst=None, rg=None, rb=None, relu=True, out=None):
    if out is None:
        out = torch.empty_like(u)
    L.check(L.lib().stgcn_ln_apply(u.data_ptr(), rows_ld(u), st.data_ptr(), g.data_ptr(), b.data_ptr(), res_mode,
                                   L.ptr(r), rows_ld(r) if r is not None else 0, L.ptr(rst), L.ptr(rg), L.ptr(rb),
                                   int(relu), out.data_ptr(), rows_ld(out), M, V, C, L.dtype_code(u.dtype),
                                   L.stream()), "ln_apply")
    return out


def ln_bwd(dy, x, st, g, b, frames, V, C, out, mask=0, mref=None, accumulate=False, dgb=None):
    """out (+)= the LayerNorm input gradient; dgb ([2][C*V] fp32, optional) += (dgamma, dbeta), reduced over the
    frames in a fixed order through a per-call workspace (stgcn_ln_bwd, ln.hip)."""
    work, nbytes = None, 0
    if dgb is not None:
        nbytes = L.lib().stgcn_ln_bwd_workspace(frames, V, C, L.dtype_code(dy.dtype))
        work = torch.empty(max(nbytes, 4) // 4, dtype=torch.float32, device=dy.device)
    L.check(L.lib().stgcn_ln_bwd(dy.data_ptr(), rows_ld(dy), mask, L.ptr(mref),
                                 rows_ld(mref) if mref is not None else 0, x.data_ptr(), rows_ld(x), st.data_ptr(),
                                 g.data_ptr(), b.data_ptr(), frames, V, C, out.data_ptr(), rows_ld(out),
                                 int(accumulate), L.ptr(dgb), L.ptr(work), nbytes, L.dtype_code(dy.dtype),
                                 L.stream()), "ln_bwd")
    return out


# ------------------------------------------------------------------------------------ head / RT
def pool_rows(x, N, R, C):
    """(N, C, 1, 1) channels-last mean over the R = T*V rows of each sample."""
    out = cl_empty(N, C, 1, 1, x.dtype, x.device)
    L.check(L.lib().stgcn_pool_rows(x.data_ptr(), rows_ld(x), N, R, C, out.data_ptr(), C, L.dtype_code(x.dtype),
                                    L.stream()), "pool_rows")
    return out


def unpool_rows(dp, R, C, M, out):
    L.check(L.lib().stgcn_unpool_rows(dp.data_ptr(), rows_ld(dp), R, C, M, out.data_ptr(), rows_ld(out),
                                      L.dtype_code(dp.dtype), L.stream()), "unpool_rows")
    return out


def box_sum(x, K, S, trans=False, out=None, accumulate=False):
    N, C, T, V = x.shape
    if out is None:
        out = cl_empty(N, C, T, V, x.dtype, x.device)
    L.check(L.lib().stgcn_box_sum(x.data_ptr(), rows_ld(x), out.data_ptr(), rows_ld(out), N, T, V, C, K, S, int(trans),
                                  int(accumulate), L.dtype_code(x.dtype), L.stream()), "box_sum")
    return out


def rt_online_step(z, fifo, acc, idx, C, V, fifo_size, S, out):
    L.check(L.lib().stgcn_rt_online_step(z.data_ptr(), fifo.data_ptr(), acc.data_ptr(), idx.data_ptr(), C, V,
                                         fifo_size, S, out.data_ptr(), L.stream()), "rt_online_step")
    return out


# ------------------------------------------------------------------------------------ AAGCN attention
def attn_scores(theta, phi, P):
    """C = softmax_w(theta_p^T phi_p) per (n, p): fp32 (N, P, V, V)."""
    N, CH, T, V = theta.shape
    C = torch.empty((N, P, V, V), dtype=torch.float32, device=theta.device)
    work = _workspace(L.lib().stgcn_attn_scores_workspace(N, T, V, P), theta.device)
    L.check(L.lib().stgcn_attn_scores(theta.data_ptr(), phi.data_ptr(), rows_ld(theta), N, T, V, P, CH // P,
                                      C.data_ptr(), work.data_ptr(), L.dtype_code(theta.dtype), L.stream()),
            "attn_scores")
    return C


def attn_proj(x, w, b):
    """theta/phi projections of a bf16 activation, fp32 out: rows (N, Nout, T, V) = w x + b (stgcn_attn_proj)."""
    N, Cin, T, V = x.shape
    Nout = w.shape[0]
    out = cl_empty(N, Nout, T, V, torch.float32, x.device)
    w = _f32c(w.reshape(Nout, Cin))
    b = None if b is None else _f32c(b)
    L.check(L.lib().stgcn_attn_proj(x.data_ptr(), rows_ld(x), N * T * V, Cin, w.data_ptr(), L.ptr(b), Nout,
                                    out.data_ptr(), Nout, L.stream()), "attn_proj")
    return out


def attn_bwd(theta, phi, P, C, dC):
    """(dtheta, dphi) as rows with theta's row stride; when theta and phi are the two halves of one row
    buffer (attn_proj's output), so are the gradients (one buffer, no concatenation downstream)."""
    N, CH, T, V = theta.shape
    dS = torch.empty_like(C)
    ld = rows_ld(theta)
    if rows_ld(phi) != ld:
        raise RuntimeError("stgcn_amd: attn_bwd needs theta and phi with the same row stride")
    es = theta.element_size()
    if ld >= 2 * CH and phi.data_ptr() - theta.data_ptr() == CH * es:
        buf = torch.empty((N, T, V, ld), dtype=theta.dtype, device=theta.device).permute(0, 3, 1, 2)
        dth, dph = buf[:, :CH], buf[:, CH:2 * CH]
    else:
        dth = torch.empty((N, T, V, ld), dtype=theta.dtype, device=theta.device).permute(0, 3, 1, 2)[:, :CH]
        dph = torch.empty((N, T, V, ld), dtype=phi.dtype, device=phi.device).permute(0, 3, 1, 2)[:, :CH]
    L.check(L.lib().stgcn_attn_bwd(theta.data_ptr(), phi.data_ptr(), rows_ld(theta), N, T, V, P, CH // P,
                                   C.data_ptr(), dC.data_ptr(), dS.data_ptr(), dth.data_ptr(), dph.data_ptr(),
                                   L.dtype_code(theta.dtype), L.stream()), "attn_bwd")
    return dth, dph


# ------------------------------------------------------------------------------ RT per-frame inference (rt_fused.hip)
def _f32c(t):
    return t if (t.dtype == torch.float32 and t.is_contiguous()) else t.float().contiguous()


def rt_frame_in(x, ln_w, ln_b, w, b):
    """(1, 3, 1, V) frame -> LayerNorm([3,1,V]) -> fcn_in: rows (1, C0, 1, V) fp32."""
    L.require_device(x)
    x = _f32c(x)
    V, C0 = x.shape[-1], w.shape[0]
    out = cl_empty(1, C0, 1, V, torch.float32, x.device)
    L.check(L.lib().stgcn_rt_frame_in(x.data_ptr(), V, _f32c(ln_w).data_ptr(), _f32c(ln_b).data_ptr(),
                                      _f32c(w).data_ptr(), _f32c(b).data_ptr(), C0, out.data_ptr(), L.stream()),
            "rt_frame_in")
    return out


def rt_frame_gcn(x, A, w, bias2d, fifo, acc, idx, wr=None):
    """Online layer conv1x1 + A-mix + FIFO step (+ residual 1x1 conv): returns (a, r) rows (1, Cout, 1, V)."""
    _, Cin, _, V = x.shape
    P = A.shape[0]
    Cout = w.shape[0] // P
    if rows_ld(x) != Cin:
        raise RuntimeError("stgcn_amd: rt_frame_gcn expects dense rows")
    a = cl_empty(1, Cout, 1, V, torch.float32, x.device)
    r = cl_empty(1, Cout, 1, V, torch.float32, x.device) if wr is not None else None
    wr_ = _f32c(wr) if wr is not None else None
    L.check(L.lib().stgcn_rt_frame_gcn(x.data_ptr(), V, Cin, Cout, P, _dense(A).data_ptr(), _f32c(w).data_ptr(),
                                       L.ptr(bias2d), fifo.data_ptr(), acc.data_ptr(), idx.data_ptr(), L.ptr(wr_),
                                       a.data_ptr(), L.ptr(r), L.stream()), "rt_frame_gcn")
    return a, r


def rt_frame_norm(a, ln_w, ln_b, res_mode, res, lnr_w, lnr_b, idx, fifo_size, S):
    """y = relu(relu(LN(a)) + res) | relu(LN(a)); advances the FIFO indices."""
    _, C, _, V = a.shape
    y = cl_empty(1, C, 1, V, torch.float32, a.device)
    L.check(L.lib().stgcn_rt_frame_norm(a.data_ptr(), _f32c(ln_w).data_ptr(), _f32c(ln_b).data_ptr(), int(res_mode),
                                        L.ptr(res), L.ptr(None if lnr_w is None else _f32c(lnr_w)),
                                        L.ptr(None if lnr_b is None else _f32c(lnr_b)), V, C, idx.data_ptr(),
                                        int(fifo_size), int(S), y.data_ptr(), L.stream()), "rt_frame_norm")
    return y


def rt_frame_out(x, w, b):
    """rows (1, C, 1, V) -> mean over V -> fcn_out: (1, K, 1)."""
    _, C, _, V = x.shape
    K = w.shape[0]
    out = torch.empty((1, K, 1), dtype=torch.float32, device=x.device)
    L.check(L.lib().stgcn_rt_frame_out(x.data_ptr(), V, C, _f32c(w).data_ptr(), L.ptr(None if b is None else _f32c(b)),
                                       K, out.data_ptr(), L.stream()), "rt_frame_out")
    return out


def rt_frame(desc, x, out):
    """The whole RT per-frame step in one launch (stgcn_rt_frame): x (1, 3, 1, V) -> out (1, K, 1); ``desc`` is
    the model's stgcn_rt_frame_desc (rtstgcn.Model._build_frame_desc) with x / out filled in here."""
    L.require_device(x)
    x = _f32c(x)
    desc.x, desc.out = x.data_ptr(), out.data_ptr()
    L.check(L.lib().stgcn_rt_frame(ctypes.byref(desc), L.stream()), "rt_frame")
    return out


# ------------------------------------------------------------------------------ window staging (window.hip)
def _capture(x):
    """(1, Cin, Lp, V) padded capture -> contiguous fp32 [Cin][Lp][V] on the device."""
    L.require_device(x)
    if x.dim() != 4 or x.shape[0] != 1:
        raise RuntimeError(f"stgcn_amd: window staging takes one (1, C, L, V) capture, got {tuple(x.shape)}")
    return _f32c(x)


def window_stats(x, W, n0, nw, mode, eps=1e-5):
    """BatchNorm1d partials (mode 0: (nb, V*Cin, 4) and nb) or LayerNorm frame statistics (mode 1: (F, 2))."""
    x = _capture(x)
    _, Cin, Lp, V = x.shape
    if mode == 0:
        nb = L.lib().stgcn_window_stat_blocks(nw, W)
        out = torch.empty((nb, V * Cin, 4), dtype=torch.float32, device=x.device)
    else:
        nb = 0
        out = torch.empty((nw + W - 1, 2), dtype=torch.float32, device=x.device)
    L.check(L.lib().stgcn_window_stats(x.data_ptr(), Cin, Lp, V, W, n0, nw, mode, eps, out.data_ptr(), L.stream()),
            "window_stats")
    return out, nb


def window_expand(x, W, n0, nw, mode, g, b, fst, w, bias, dtype):
    """First activation of windows [n0, n0+nw): logical (nw, Cout, W, V) channels-last rows."""
    x = _capture(x)
    _, Cin, Lp, V = x.shape
    Cout = w.shape[0]
    out = cl_empty(nw, Cout, W, V, dtype, x.device)
    L.check(L.lib().stgcn_window_expand(x.data_ptr(), Cin, Lp, V, W, n0, nw, mode, _f32c(g).data_ptr(),
                                        _f32c(b).data_ptr(), L.ptr(fst), _f32c(w).data_ptr(),
                                        L.ptr(None if bias is None else _f32c(bias)), Cout, out.data_ptr(), Cout,
                                        L.dtype_code(dtype), L.stream()), "window_expand")
    return out


def window_grad(dy, x, W, n0, nw, mode, st, gamma, beta, w):
    """(dgamma, dbeta, dw [Cout][Cin], db) of the staged first activation from its gradient rows."""
    x = _capture(x)
    _, Cin, Lp, V = x.shape
    Cout = w.shape[0]
    dev = x.device
    work = _workspace(L.lib().stgcn_window_grad_workspace(nw, W, V, Cin, Cout), dev)
    dg = torch.empty(V * Cin, dtype=torch.float32, device=dev)
    dbeta = torch.empty(V * Cin, dtype=torch.float32, device=dev)
    dw = torch.empty((Cout, Cin), dtype=torch.float32, device=dev)
    db = torch.empty(Cout, dtype=torch.float32, device=dev)
    L.check(L.lib().stgcn_window_grad(dy.data_ptr(), rows_ld(dy), L.dtype_code(dy.dtype), x.data_ptr(), Cin, Lp, V, W,
                                      n0, nw, mode, _f32c(st).data_ptr(), _f32c(gamma).data_ptr(),
                                      _f32c(beta).data_ptr(), _f32c(w).data_ptr(), Cout, work.data_ptr(),
                                      dg.data_ptr(), dbeta.data_ptr(), dw.data_ptr(), db.data_ptr(), L.stream()),
            "window_grad")
    return dg, dbeta, dw, db

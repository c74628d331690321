"""ctypes binding of libstgcn_amd.so (the C-ABI declared in include/stgcn_amd.h).

The library is the ONLY compute path of this package: there is no CPU or eager-PyTorch
fallback.  If the shared object is missing, or no HIP device is visible, every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("STGCN_LIB") or os.path.join(_HERE, "lib", "libstgcn_amd.so")  # STGCN_LIB: A/B builds

# the STGCN_ABI_VERSION of include/stgcn_amd.h these bindings mirror (test_cpu_host checks the two agree)
ABI_VERSION = 5

_ERR = {1: "bad shape/arguments", 2: "unsupported dtype", 3: "HIP launch error"}

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_long = ctypes.c_long
c_float = ctypes.c_float


class AdamEntry(ctypes.Structure):
    _fields_ = [("p", c_void_p), ("m", c_void_p), ("v", c_void_p), ("n", c_long), ("b0", c_long), ("vec", c_int),
                ("pad_", c_int)]


class ConvDesc(ctypes.Structure):
    _fields_ = [("in_", c_void_p), ("out", c_void_p), ("w", c_void_p), ("bias", c_void_p), ("pro_a", c_void_p),
                ("pro_b", c_void_p), ("pro_stats", c_void_p), ("stats", c_void_p)] + \
               [(n, c_int) for n in ("N", "T_in", "T_out", "V", "Cin", "Cout", "Cin_pad", "Cout_pad", "Kt", "stride",
                                     "pad", "trans", "pro", "bias_mode", "accumulate", "in_ld", "out_ld")] + \
               [("w_frag", c_void_p)]


class WgradDesc(ctypes.Structure):
    _fields_ = [("in_", c_void_p), ("dy", c_void_p), ("dw", c_void_p), ("pro_a", c_void_p), ("pro_b", c_void_p),
                ("pro_stats", c_void_p)] + \
               [(n, c_int) for n in ("N", "T_in", "T_out", "V", "Cin", "Cout", "Kt", "stride", "pad", "pro",
                                     "in_ld", "dy_ld")] + [("rows_per_block", c_long), ("work", c_void_p),
                                                           ("work_bytes", c_long), ("out_mode", c_int), ("pad_", c_int)]


class AmixDesc(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("out", c_void_p), ("A", c_void_p)] + \
               [(n, c_int) for n in ("N", "T", "V", "P", "Cin", "per_sample", "accumulate", "x_ld", "out_ld")]


class GconvDesc(ctypes.Structure):
    _fields_ = [("in_", c_void_p), ("out", c_void_p), ("w", c_void_p), ("nbr", c_void_p), ("deg", c_void_p),
                ("bias", c_void_p), ("stats", c_void_p)] + \
               [(n, c_int) for n in ("NT", "V", "J", "Cin", "Cout", "Cin_pad", "Cout_pad", "in_ld", "out_ld",
                                     "accumulate")] + [("res", c_void_p), ("res_bits", c_void_p), ("res_ld", c_int)]


class GconvWgradDesc(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("dy", c_void_p), ("nbr", c_void_p), ("deg", c_void_p), ("dweff", c_void_p)] + \
               [(n, c_int) for n in ("NT", "V", "J", "Cin", "Cout", "x_ld", "dy_ld")] + \
               [("work", c_void_p), ("work_bytes", c_long), ("rowsum", c_void_p), ("phase", c_int), ("pad_", c_int)]


class LayerFusedDesc(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("x", "z", "wg_frag", "A", "gbias", "wt_frag", "tbias")] + \
               [(n, c_int) for n in ("N", "T", "V", "P", "x_ld", "z_ld")] + \
               [(n, c_void_p) for n in ("ln1_g", "ln1_b", "ln2_g", "ln2_b")] + [("residual", c_int), ("pad_", c_int)] + \
               [(n, c_void_p) for n in ("g_out", "u_out", "st1_out", "st2_out")] + [("g_ld", c_int), ("u_ld", c_int)] + \
               [("h_out", c_void_p), ("h_ld", c_int), ("pad2_", c_int)]


class BnBwdDesc(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("dy", "mref", "x1", "x2", "msc", "msh", "mean_rstd1", "mean_rstd2",
                                        "gamma1", "gamma2", "sums", "out1", "out2", "osum", "work")] + \
               [("M", c_long)] + [(n, c_int) for n in ("C", "mask", "lddy", "ldm", "ldx1", "ldx2", "ldo1", "ldo2",
                                                       "acc2")]


class PrepJob(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("kind", "dtype", "trans", "Kt", "Co", "Ci", "cp", "kp")] + \
               [(n, c_long) for n in ("s0", "s1", "s2", "threads")] + \
               [(n, c_void_p) for n in ("src", "dst", "dst_frag", "A", "M", "nbr", "deg")] + \
               [(n, c_int) for n in ("P", "V", "J", "R_pad", "C_pad", "pad_")] + \
               [(n, c_void_p) for n in ("bconv", "bias2d")]


RT_MAX_LAYERS = 12  # STGCN_RT_MAX_LAYERS


class RtLayer(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("Cin", "Cout", "P", "fifo_size", "S", "res_mode")] + \
               [(n, c_void_p) for n in ("A", "w", "bias2d", "wr", "ln_w", "ln_b", "lnr_w", "lnr_b", "fifo", "acc",
                                        "idx", "a_buf", "r_buf")]


class RtFrameDesc(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("V", "L", "C0", "K", "blocks")] + \
               [(n, c_void_p) for n in ("x", "ln_w", "ln_b", "w_in", "b_in", "w_out", "b_out", "out", "sync",
                                        "status")] + \
               [("layers", RtLayer * RT_MAX_LAYERS)]


# name -> (restype, argtypes)
_SIGS = {
    "stgcn_abi_version": (c_int, []),
    "stgcn_conv_rows": (c_int, [ctypes.POINTER(ConvDesc), c_int, c_void_p]),
    "stgcn_conv_rows_col_tile": (c_int, [c_int]),
    "stgcn_conv_rows_row_blocks": (c_long, [c_long, c_int]),
    "stgcn_conv_wgrad": (c_int, [ctypes.POINTER(WgradDesc), c_int, c_void_p]),
    "stgcn_conv_wgrad_workspace": (c_long, [ctypes.POINTER(WgradDesc), c_int]),
    "stgcn_gconv": (c_int, [ctypes.POINTER(GconvDesc), c_int, c_void_p]),
    "stgcn_bn_bwd_fused_workspace": (c_long, [c_long, c_int, c_int]),
    "stgcn_bn_bwd_fused_reduce": (c_int, [ctypes.POINTER(BnBwdDesc), c_int, c_void_p]),
    "stgcn_bn_bwd_fused_apply": (c_int, [ctypes.POINTER(BnBwdDesc), c_int, c_void_p]),
    "stgcn_gconv_row_blocks": (c_long, [c_int, c_int]),
    "stgcn_gconv_weights_bias": (c_int, [c_void_p] * 5 + [c_int] * 5 + [c_void_p, c_int, c_int, c_void_p, c_int,
                                                                       c_void_p]),
    "stgcn_gconv_weights": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 6 + [c_void_p, c_int, c_int,
                                                                                           c_int, c_void_p]),
    "stgcn_gconv_wgrad": (c_int, [ctypes.POINTER(GconvWgradDesc), c_int, c_void_p]),
    "stgcn_gconv_wgrad_workspace": (c_long, [ctypes.POINTER(GconvWgradDesc), c_int]),
    "stgcn_gconv_wgrad_finish_workspace": (ctypes.c_long, [c_int] * 5),
    "stgcn_gconv_wgrad_finish": (c_int, [c_void_p] * 5 + [c_int] * 5 + [c_void_p, c_void_p, c_void_p, c_void_p]),
    "stgcn_gconv_wgrad_finish_bias": (c_int, [c_void_p] * 5 + [c_int] * 5 + [c_void_p] * 7),
    "stgcn_amix_fwd": (c_int, [ctypes.POINTER(AmixDesc), c_int, c_void_p]),
    "stgcn_amix_trans": (c_int, [ctypes.POINTER(AmixDesc), c_int, c_void_p]),
    "stgcn_gcn_bias_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "stgcn_pack_weight": (c_int, [c_void_p, ctypes.c_long, ctypes.c_long, ctypes.c_long, c_int, c_int, c_int,
                                  c_void_p, c_int, c_int, c_int, c_void_p]),
    "stgcn_tconv_frame": (c_int, [ctypes.POINTER(ConvDesc), c_void_p]),
    "stgcn_tconv_frame_row_blocks": (ctypes.c_long, [c_int, c_int]),
    "stgcn_pack_weight_s2frag": (c_int, [c_void_p, ctypes.c_long, ctypes.c_long, ctypes.c_long, c_int, c_int,
                                         c_void_p, c_int, c_int, c_void_p]),
    "stgcn_pack_weight_frag": (c_int, [c_void_p, ctypes.c_long, ctypes.c_long, ctypes.c_long, c_int, c_int, c_int,
                                       c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "stgcn_amix_dA_workspace": (ctypes.c_long, [ctypes.POINTER(AmixDesc)]),
    "stgcn_amix_dA": (c_int, [ctypes.POINTER(AmixDesc), c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "stgcn_gcn_bias": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "stgcn_bn_stat_blocks": (c_long, [c_long]),
    "stgcn_bn_stats_partial": (c_int, [c_void_p, c_int, c_long, c_int, c_void_p, c_int, c_void_p]),
    "stgcn_bn_finalize": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                  c_void_p, c_void_p]),
    "stgcn_bn_merge": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "stgcn_bn_apply": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p,
                               c_int, c_void_p, c_int, c_long, c_int, c_int, c_void_p]),
    "stgcn_bn_apply_bits": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                    c_int, c_void_p, c_int, c_long, c_int, c_void_p, c_void_p]),
    "stgcn_bn_bwd_reduce": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                    c_void_p, c_long, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "stgcn_bn_bwd_apply": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                   c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p, c_int, c_int, c_int,
                                   c_void_p]),
    "stgcn_rowgroup_sum": (c_int, [c_void_p, c_int, c_long, c_int, c_int, c_long, c_void_p, c_void_p, c_int,
                                   c_void_p]),
    "stgcn_rowgroup_sum_workspace": (c_long, [c_long, c_int, c_int, c_long]),
    "stgcn_ln_stats": (c_int, [c_void_p, c_int, c_long, c_int, c_int, c_float, c_void_p, c_int, c_void_p]),
    "stgcn_ln_apply": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p,
                               c_void_p, c_void_p, c_int, c_void_p, c_int, c_long, c_int, c_int, c_int, c_void_p]),
    "stgcn_ln_bwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                             c_long, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_long, c_int,
                             c_void_p]),
    "stgcn_ln_bwd_workspace": (c_long, [c_long, c_int, c_int, c_int]),
    "stgcn_cast_colsum": (c_int, [c_void_p, c_int, c_long, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "stgcn_cast_colsum_workspace": (c_long, [c_long, c_int]),
    "stgcn_pool_rows": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
    "stgcn_unpool_rows": (c_int, [c_void_p, c_int, c_int, c_int, c_long, c_void_p, c_int, c_int, c_void_p]),
    "stgcn_box_sum": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_int, c_void_p]),
    "stgcn_rt_online_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                     c_void_p]),
    "stgcn_attn_scores_workspace": (ctypes.c_long, [c_int, c_int, c_int, c_int]),
    "stgcn_attn_scores": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                  c_int, c_void_p]),
    "stgcn_attn_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "stgcn_layer_fused_fwd": (c_int, [ctypes.POINTER(LayerFusedDesc), c_void_p]),
    "stgcn_rt_frame_in": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "stgcn_rt_frame_gcn": (c_int, [c_void_p, c_int, c_int, c_int, c_int] + [c_void_p] * 10),
    "stgcn_rt_frame_norm": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                    c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "stgcn_rt_frame_out": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "stgcn_rt_frame": (c_int, [ctypes.POINTER(RtFrameDesc), c_void_p]),
    "stgcn_window_stat_blocks": (c_int, [c_int, c_int]),
    "stgcn_window_stats": (c_int, [c_void_p] + [c_int] * 7 + [c_float, c_void_p, c_void_p]),
    "stgcn_window_expand": (c_int, [c_void_p] + [c_int] * 7 + [c_void_p] * 5 + [c_int, c_void_p, c_int, c_int,
                                                                                c_void_p]),
    "stgcn_window_grad_workspace": (ctypes.c_long, [c_int] * 5),
    "stgcn_window_grad": (c_int, [c_void_p, c_int, c_int, c_void_p] + [c_int] * 7 + [c_void_p] * 4 + [c_int] +
                          [c_void_p] * 6),
    "stgcn_attn_proj": (c_int, [c_void_p, c_int, c_long, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "stgcn_segment_metrics_workspace": (ctypes.c_long, [c_int]),
    "stgcn_segment_metrics": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p]),
    "stgcn_seg_loss_workspace": (ctypes.c_long, [c_int]),
    "stgcn_seg_loss": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                               c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "stgcn_seg_loss_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p]),
    "stgcn_prep_check": (c_int, [ctypes.POINTER(PrepJob), c_int]),
    "stgcn_prep_run": (c_int, [c_void_p, c_void_p, c_int, c_long, c_void_p]),
    "stgcn_adam_blocks": (ctypes.c_long, [c_long]),
    "stgcn_adam_step": (c_int, [c_void_p, c_int, c_long, c_void_p, c_void_p] + [ctypes.c_double] * 5 + [c_void_p]),
}

EXPORTS = tuple(_SIGS)

_lib = None


def load_library(path: str = LIB_PATH):
    """Load the shared object and bind every exported symbol (raises if anything is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"stgcn_amd: native library not built: {path} (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)  # AttributeError if the symbol is missing
        fn.restype = res
        fn.argtypes = args
    got = lib.stgcn_abi_version()
    if got != ABI_VERSION:
        raise RuntimeError(f"stgcn_amd: {path} implements C-ABI version {got}, these bindings need {ABI_VERSION} "
                           "(stale build: run __graft_entry__.build())")
    _lib = lib
    return lib


def lib():
    if _lib is None:
        load_library()
    return _lib


def check(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"stgcn_amd.{name} failed with code {rc} ({_ERR.get(rc, 'unknown')})")


def require_device(t: torch.Tensor):
    if not t.is_cuda:
        raise RuntimeError("stgcn_amd ops run on the HIP device only (no CPU fallback); got a CPU tensor")


def stream() -> int:
    """Raw handle of the current device's current stream (what torch.cuda.current_stream().cuda_stream
    returns, without building a Stream object: 0.1 vs 2.6 us per call, and every kernel wrapper calls it)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return 0
    if dt == torch.bfloat16:
        return 1
    raise RuntimeError(f"stgcn_amd: unsupported dtype {dt} (fp32 or bf16)")


def ptr(t):
    return None if t is None else t.data_ptr()

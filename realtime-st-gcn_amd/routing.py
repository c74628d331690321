"""Kernel-routing switches of the package, in one place.

Every switch only chooses between kernels that compute the same result (each route is covered by the -m gpu
suite); none changes numerics beyond the rounding order of its kernels.  Defaults are the measured-fastest
routes on MI355X.  The environment variables are read once at import; code (tests, tools) may
also assign the attributes directly.

    side_stream         STGCN_SIDE_STREAM=1   weight-gradient branch of a layer backward (and the residual branch
                                              of the forward) on a per-device side stream (default off: with
                                              the one-launch weight preparation the config-2 step measured 8.59
                                              ms on one stream vs 8.72 with the side stream, same box)
    fused_inference     STGCN_FUSED=0         no_grad forward of 64->64 stride-1 layers through the fused layer
                                              kernel layer_fused.hip (default on for LayerNorm layers)
    fused_bn_inference  STGCN_FUSED_BN=0      BatchNorm layers too (default on since the fused kernel reached 78-82 us:
                                              the two-pass fused forward measured 0.175 vs 0.187 ms graph-replayed,
                                              0.178 vs 0.179 eager)
    fused_ln_train      STGCN_FUSED_LN_TRAIN=1  training forward of LayerNorm 64->64 stride-1 layers through the same
                                              one-kernel layer (it also writes g, u and both LN statistics for the
                                              unfused backward).  Default off since the LayerNorm kernels of ln.hip:
                                              the LN training step measured 8.77 ms unfused vs 8.86 fused (r04k)
    gcn_tile            STGCN_GCN_TILE=0|1|auto  graph conv on the two-stage MFMA kernel gcn_tile.hip (default 0)
    gcn_afirst          STGCN_GCN_AFIRST=1    force the A-first graph conv (amix + GEMM) for shared graphs
    gcn_afirst_min_c    STGCN_GCN_AFIRST_MIN_C=<C>  ... only for layers with at least C input channels (A/B of the
                                              A-first form where the gathered form's per-joint effective weights
                                              outgrow L2; default 0 = off)
    gconv_wgrad_frame   STGCN_GWF=1           graph-conv weight / adjacency / bias gradients (bf16, shared A) in the
                                              one-pass frame kernel gconv_wgrad_frame.hip instead of the per-joint
                                              dWeff kernel + finish (default off: 115 vs 72 us at C = 64, 242 vs 133
                                              at C = 256 in isolation, r04c)
    gcn_frame           STGCN_GCN_FRAME=1     graph conv forward / data grad (bf16, shared A, 64 or 128 kernel-input
                                              channels) on the frame-streaming kernel gcn_frame.hip instead of the
                                              joint-gathered gconv.hip (default off: equal forward, slower data
                                              grad in isolation, r04c)
    tconv_frame         STGCN_TCONV_FRAME=1   64-channel Kt = 9 stride-1 temporal conv forward (BatchNorm layers) on the
                                              frame-streaming kernel tconv_frame.hip instead of conv_wide (default off:
                                              67.1 vs 64.1 us in isolation, r04d)
    tconv_frame_dgrad   STGCN_TCONV_FRAME_DGRAD=0  its data grad on tconv_frame.hip instead of conv_persist (default on:
                                              52.0 vs 65.0 us in isolation, r04d)
    prep_plan           STGCN_PREP_PLAN=0     stgcn.Model training forwards pack every weight per call instead of
                                              in the one-launch plan (native.PrepPlan; default on)
"""
import os


class _Routing:
    def __init__(self):
        e = os.environ.get
        self.side_stream = e("STGCN_SIDE_STREAM", "0") == "1"
        self.fused_inference = e("STGCN_FUSED", "1") != "0"
        self.fused_bn_inference = e("STGCN_FUSED_BN", "1") != "0"
        self.fused_ln_train = e("STGCN_FUSED_LN_TRAIN", "0") == "1"
        self.gcn_tile = e("STGCN_GCN_TILE", "0")
        self.gcn_afirst = e("STGCN_GCN_AFIRST", "0") not in ("0", "")
        self.gcn_afirst_min_c = int(e("STGCN_GCN_AFIRST_MIN_C", "0") or 0)
        self.prep_plan = e("STGCN_PREP_PLAN", "1") != "0"
        self.gconv_wgrad_frame = e("STGCN_GWF", "0") == "1"
        self.gcn_frame = e("STGCN_GCN_FRAME", "0") == "1"
        self.tconv_frame = e("STGCN_TCONV_FRAME", "0") == "1"
        self.tconv_frame_dgrad = e("STGCN_TCONV_FRAME_DGRAD", "1") != "0"


ROUTING = _Routing()

"""Kernel-routing switches of the package, in one place.

Every switch only chooses between kernels that compute the same result (each route is covered by the -m gpu
suite); none changes numerics beyond the rounding order of its kernels.  Defaults are the measured-fastest
routes on MI355X.  The environment variables are read once at import; code (tests, tools) may
also assign the attributes directly.

    fused_inference     STGCN_FUSED=0         no_grad forward of LayerNorm 64->64 stride-1 layers through the one-kernel
                                              layer layer_fused.hip (default on: 0.126 vs 0.208 ms unfused)
    fused_bn_inference  STGCN_FUSED_BN=1      BatchNorm layers too (default OFF: the two-pass fused forward loses on the
                                              driver's boxes, BENCH_r04 0.1757 vs 0.1657 ms eager / 0.1725 vs 0.1709
                                              graph-replayed, r05a 0.1758 vs 0.1664 / 0.1741 vs 0.1714)
    fused_ln_train      STGCN_FUSED_LN_TRAIN=0  training forward of LayerNorm 64->64 stride-1 layers through the same
                                              one-kernel layer (it also writes g, u, h and both LN statistics for the
                                              unfused backward).  Default on since round 5 (frame-aligned LN2
                                              epilogue, h written by the kernel, packs from the prep launch): LN
                                              training step 8.397-8.430 fused vs 8.442-8.456 ms unfused (r05, 3
                                              interleaved runs; round 4: 8.86 vs 8.77)
    bn_mask_bits        STGCN_BN_BITS=0       the BatchNorm-2 backward reads the forward output's sign bits (written by bn_apply)
                                              for its ReLU mask instead of the output itself (default on)
    bn_tcn_fused        STGCN_BN_TCN=1        training forward of BatchNorm 64->64 stride-1 layers: the temporal conv through
                                              layer_fused.hip's g-input mode instead of conv_wide (default OFF since
                                              round 6: step-neutral, 7.513 vs 7.513 ms, and it moved the most
                                              downstream bf16 gradient)
    prep_plan           STGCN_PREP_PLAN=0     stgcn.Model training forwards pack every weight per call instead of
                                              in the one-launch plan (native.PrepPlan; default on)

Routes removed in round 5 after losing their A/Bs (last measurements in DESIGN 4.4 / 4.11 / 3): the frame-streaming
graph conv (gcn_frame.hip: equal forward, slower data gradient) and graph-conv weight gradient
(gconv_wgrad_frame.hip: 115 vs 72 us at C = 64), gcn_tile.hip as the training graph conv (equal inside the step;
it remains pass 1 of the fused BatchNorm form), the tconv_frame.hip forward (67.1 vs 64.1 us; its data gradient
ships), the weight-gradient side stream (8.68 vs 8.55 ms/step) and the forced A-first graph conv for shared graphs.
"""
import os


class _Routing:
    def __init__(self):
        e = os.environ.get
        self.fused_inference = e("STGCN_FUSED", "1") != "0"
        self.fused_bn_inference = e("STGCN_FUSED_BN", "0") == "1"
        self.fused_ln_train = e("STGCN_FUSED_LN_TRAIN", "1") != "0"
        self.bn_mask_bits = e("STGCN_BN_BITS", "1") != "0"
        self.bn_tcn_fused = e("STGCN_BN_TCN", "0") == "1"
        self.prep_plan = e("STGCN_PREP_PLAN", "1") != "0"


ROUTING = _Routing()

"""Kernel-routing switches of the package, in one place.

Every switch only chooses between kernels that compute the same result (each route is covered by the -m gpu
suite); none changes numerics beyond the rounding order of its kernels.  Defaults are the measured-fastest
routes on MI355X.  The environment variables are read once at import; code (tests, tools) may
also assign the attributes directly.

    fused_inference     STGCN_FUSED=0         no_grad forward of LayerNorm 64->64 stride-1 layers through the one-kernel
                                              layer layer_fused.hip (default on: 0.126 vs 0.208 ms unfused)
    fused_ln_train      STGCN_FUSED_LN_TRAIN=0  training forward of LayerNorm 64->64 stride-1 layers through the same
                                              one-kernel layer (it also writes g, u, h and both LN statistics for the
                                              unfused backward).  Default on since round 5 (frame-aligned LN2
                                              epilogue, h written by the kernel, packs from the prep launch): LN
                                              training step 8.397-8.430 fused vs 8.442-8.456 ms unfused (r05, 3
                                              interleaved runs; round 4: 8.86 vs 8.77)
    bn_mask_bits        STGCN_BN_BITS=0       the BatchNorm-2 backward reads the forward output's sign bits (written by bn_apply)
                                              for its ReLU mask instead of the output itself (default on)
    rt_one_launch       STGCN_RT_ONE_LAUNCH=0 per-frame RT-ST-GCN inference (LayerNorm, config 3) as ONE persistent launch with
                                              in-launch grid barriers (stgcn_rt_frame) instead of 2 launches per layer
                                              (default on)
    prep_plan           STGCN_PREP_PLAN=0     stgcn.Model training forwards pack every weight per call instead of
                                              in the one-launch plan (native.PrepPlan; default on)

Routes removed in round 6: the BatchNorm two-pass fused inference form (gcn_tile.hip pass 1 + layer_fused.hip pass 2;
it lost to the unfused forward on every driver box: BENCH_r05 0.1736 vs 0.1677 ms) and layer_fused.hip's g-input
temporal conv for the BatchNorm training forward (step-neutral, 7.513 vs 7.513 ms).
Routes removed in round 5 after losing their A/Bs (last measurements in DESIGN 4.4 / 4.11 / 3): the frame-streaming
graph conv (gcn_frame.hip: equal forward, slower data gradient) and graph-conv weight gradient
(gconv_wgrad_frame.hip: 115 vs 72 us at C = 64), gcn_tile.hip as the training graph conv (equal inside the step), the tconv_frame.hip forward (67.1 vs 64.1 us; its data gradient
ships), the weight-gradient side stream (8.68 vs 8.55 ms/step) and the forced A-first graph conv for shared graphs.
Tried in round 6 and not kept: only the graph-conv weight gradient's latency-bound tail (slab reduction + dW / dA / db
finish, ~33 us per layer) on a second stream beside the layer's graph-conv data gradient — 8.28 / 7.88 / 7.85 vs
7.63 / (8.74) / 7.63 ms/step (interleaved, one box): co-running still slows the data gradient more than it hides.
"""
import os


class _Routing:
    def __init__(self):
        e = os.environ.get
        self.fused_inference = e("STGCN_FUSED", "1") != "0"
        self.fused_ln_train = e("STGCN_FUSED_LN_TRAIN", "1") != "0"
        self.bn_mask_bits = e("STGCN_BN_BITS", "1") != "0"
        self.prep_plan = e("STGCN_PREP_PLAN", "1") != "0"
        self.rt_one_launch = e("STGCN_RT_ONE_LAUNCH", "1") != "0"


ROUTING = _Routing()

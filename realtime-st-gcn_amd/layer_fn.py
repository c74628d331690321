"""Forward/backward of one ST-GCN layer as a sequence of HIP kernel launches.

StgcnLayer.forward (models/stgcn/stgcn.py:181-193) is

    res = identity(x) | norm_r(conv1x1_s(x)) | 0
    g   = ConvTemporalGraphical(x, A)                 tgcn.py:58-79   (1x1 conv -> @A -> sum_P)
    u   = conv_Kt_s(relu(norm1(g)))                    stgcn.py:151-159
    y   = relu(norm2(u) + res)                         stgcn.py:160,193

with norm = BatchNorm2d(track_running_stats=False) or the custom LayerNorm([C,1,V]).

Kernel schedule (forward, BatchNorm):
  amix_fwd(x, A)                -> XA                     (A applied first, exact)
  gcn_bias(A, b)                -> bias2d[V][C]
  conv_rows(XA, Wg, bias2d)     -> g   + BN1 partial stats (epilogue)
  bn_finalize                   -> scale1/shift1
  conv_rows(g, Wt, pro=BN1+ReLU)-> u   + BN2 partial stats (prologue applies norm1+ReLU on load)
  [conv_rows(x, Wr, s) -> r + stats ; finalize]
  bn_finalize, bn_apply(u, +res, ReLU) -> y
Backward mirrors it with the transposed convs (conv_rows trans=1), the m-reduction weight-grad
kernel (conv_wgrad), the BN reduce/apply pair, amix_trans / amix_dA for the graph part.
Everything is a HIP kernel of libstgcn_amd.so; the only torch work here is allocation, weight
re-packing (tiny tensors) and the (P x V)-sized reshuffles of the A/bias gradients.
"""
from __future__ import annotations

import torch

from . import native as K
from .routing import ROUTING
from .syncbn import active_sync

BN, LN = "BatchNorm", "LayerNorm"

def _flat_ln(p):
    """LayerNorm([C,1,V]) parameter (C,1,V) -> flat fp32 [C*V] indexed c*V+v (kernel convention)."""
    return p.detach().reshape(-1).float().contiguous()


def gcn_forward(x, A32, wg, bg, dtype, stats=None):
    """ConvTemporalGraphical forward on rows: XA = A-mix(x); g = XA @ Wg' + bias2d.  Returns (XA, g, cp)."""
    N, Cin, T, V = x.shape
    P = A32.shape[-3]
    Cout = wg.shape[0] // P
    XA = K.amix_fwd(x, A32)
    wg3 = wg.detach().float().view(P, Cout, Cin).permute(1, 0, 2).reshape(1, Cout, P * Cin)
    wgp, cp, kp = K.pack_weight(wg3, dtype)
    bias2d = K.gcn_bias(A32, bg.detach().float().contiguous(), N, Cout)
    g = K.conv_rows(XA, wgp, P * Cin, Cout, cp, kp, T, T, bias=bias2d, bias_mode=3 if A32.dim() == 4 else 2,
                    stats=stats)
    return XA, g, cp


def gcn_stats_buffer(M, Cout, dev):
    cp = -(-Cout // K.col_tile(Cout)) * K.col_tile(Cout)
    return torch.zeros((K.row_blocks(M, Cout), cp, 4), dtype=torch.float32, device=dev), cp


def gcn_backward(x, A32, XA, wg, bg, dg, dx, accumulate, dtype):
    """Backward of gcn_forward given dg: dx (+)= A^T-mix(dg @ Wg), returns (dA fp32, dWg, dbg)."""
    N, Cin, T, V = x.shape
    P = A32.shape[-3]
    Cout = wg.shape[0] // P
    M = N * T * V
    wgT = wg.detach().float().view(P, Cout, Cin).permute(0, 2, 1).reshape(1, P * Cin, Cout)
    wgTp, cq, kq = K.pack_weight(wgT, dtype)
    DW = K.conv_rows(dg, wgTp, Cout, P * Cin, cq, kq, T, T)
    K.amix_trans(DW, A32, Cin, dx, accumulate=accumulate)
    dA = K.amix_dA(x, DW, A32)
    bgp = bg.detach().float().view(P, Cout)
    # the conv bias pushed through A: dA[p][v][w] += sum_c b_p[c] S[w][c] (independent of v)
    if A32.dim() == 4:
        Sn = K.rowgroup_sum(dg, M, Cout, V, per_sample=True)            # [N][V(w)][Cout]
        dA += torch.einsum("pc,nwc->npw", bgp, Sn).unsqueeze(2)
        dbg = torch.einsum("npw,nwc->pc", A32.sum(dim=2), Sn).reshape(-1)
    else:
        S = K.rowgroup_sum(dg, M, Cout, V)                               # [V(w)][Cout]
        dA += (bgp @ S.t()).unsqueeze(1)
        dbg = (A32.sum(dim=1) @ S).reshape(-1)
    dwg = K.conv_wgrad(XA, dg, P * Cin, Cout, T, T, Kt=1)                # [1][Cout][P*Cin]
    dwg = dwg.view(Cout, P, Cin).permute(1, 0, 2).reshape(P * Cout, Cin, 1, 1)
    return dA, dwg, dbg


def _packs(cache, wg, wt, P, Cin, Cout, dtype):
    """Packed graph-conv (the fused layer's W' image) and temporal-conv (fragment image) weights, reused while the
    parameters are unchanged (keyed by storage and in-place version): inference packs once."""
    key = (wg.data_ptr(), wg._version, wt.data_ptr(), wt._version, dtype)
    if cache is not None and cache.get("key") == key:
        return cache["val"]
    wgf = wg.detach().float().view(P, Cout, Cin).permute(1, 0, 2).reshape(Cout, P * Cin)
    wimg, cpg, kwg = K.pack_gcn_weight(wgf, dtype)
    wt3 = wt.detach().float().squeeze(-1).permute(2, 0, 1)  # [Kt][Cout][Cin]
    wtp, _, _ = K.pack_weight(wt3, dtype, stride=1)
    val = (wimg, cpg, kwg, wtp)
    if cache is not None:
        cache["key"], cache["val"] = key, val
    return val


class LayerPacks:
    """Packed operands of one StgcnLayer's training step, filled by the model's PrepPlan launch
    (native.PrepPlan): graph-conv effective weights + bias through A (forward), their data-gradient form,
    temporal conv (forward / data gradient) and residual 1x1 conv (forward / data gradient) packs, each as
    the (tensor, Cout_pad, Cin_pad) triple pack_weight returns (gw: (weights, bias2d))."""
    __slots__ = ("gw", "gwT", "wt", "wtT", "wr", "wrT")

    def __init__(self):
        self.gw = self.gwT = self.wt = self.wtT = self.wr = self.wrT = None


def plan_layer_packs(plan, layer, A, M, dtype):
    """Record in ``plan`` every pack StgcnLayerFunction builds per call for ``layer`` fed ``A * M`` (the
    model's graph and the layer's edge importance, M None without importance); None when the layer takes a
    route that packs differently (per-sample or dense A: the A-first graph conv)."""
    sup = layer._gsup
    P, V = A.shape[0], A.shape[-1]
    conv = layer.tcn[2]
    Cout, Cin = conv.out_channels, layer.gcn.conv.in_channels
    kt, stride = layer.kernel_size[0], layer.stride
    if sup is None or A.dim() != 3 or sup.dense(P):
        return None
    pk = LayerPacks()
    wg2 = layer.gcn.conv.weight.detach().reshape(P * Cout, Cin)
    pk.gw = K.gconv_weights(A, wg2, sup, Cout, Cin, False, dtype, bias=layer.gcn.conv.bias.detach(), plan=plan, M=M)
    pk.gwT = K.gconv_weights(A, wg2, sup, Cout, Cin, True, dtype, plan=plan, M=M)
    wt = conv.weight.detach().squeeze(-1)
    pk.wt = K.pack_weight(wt.permute(2, 0, 1), dtype, stride=stride, plan=plan)
    pk.wtT = K.pack_weight(wt.permute(2, 1, 0), dtype, stride=stride, trans=True, plan=plan)
    if layer.is_residual_conv:
        wr = layer.residual[0].weight.detach().view(Cout, Cin)
        pk.wr = K.pack_weight(wr.unsqueeze(0), dtype, plan=plan)
        pk.wrT = K.pack_weight(wr.t().unsqueeze(0), dtype, plan=plan)
    return pk


def fused_layer_forward(x, A32, wg, bg, n1w, n1b, wt, bt, n2w, n2b, residual, dtype, tag=None, cache=None,
                        train=False, packs=None):
    """StgcnLayer.forward (stgcn.py:181-193) of a LayerNorm layer through layer_fused.hip: both norms are per frame,
    so the whole layer is one kernel (g and h stay on chip).  ``train``: the kernel also writes what the unfused
    backward reads and this returns (y, g, u, ls1, ls2, h).  x: channels-last bf16 (N, 64, T, V).  ``packs``: the
    step's LayerPacks (training): the temporal-conv fragment image and the bias through A come from the model's one
    prep launch instead of per-layer launches."""
    N, Cin, T, V = x.shape
    P = A32.shape[0]
    Cout = wt.shape[0]
    if packs is not None and packs.wt is not None and packs.gw is not None:
        bias2d = packs.gw[1]
        wgf = wg.detach().float().view(P, Cout, Cin).permute(1, 0, 2).reshape(Cout, P * Cin)
        wimg, cpg, kwg = K.pack_gcn_weight(wgf, dtype)
        wtp = packs.wt[0]
    else:
        bias2d = K.gcn_bias(A32, bg.detach().float().contiguous(), N, Cout)
        wimg, cpg, kwg, wtp = _packs(cache, wg, wt, P, Cin, Cout, dtype)
    # the LayerNorm([64,1,V]) parameters as per-joint [V][64] rows, re-laid-out when one changed (every training
    # step): one stacking launch for the four (the kernel reads 16-B channel runs per joint)
    lkey = tuple((t.data_ptr(), t._version) for t in (n1w, n1b, n2w, n2b))
    if cache is not None and cache.get("ln_key") == lkey:
        ln = cache["ln_val"]
    else:
        ln = tuple(torch.stack([p.detach().float().reshape(Cout, V).t() for p in (n1w, n1b, n2w, n2b)]).unbind(0))
        if cache is not None:
            cache["ln_key"], cache["ln_val"] = lkey, ln
    return K.layer_fused(x, A32, wimg, bias2d, wtp, bt.detach().float().contiguous(), ln, tag=tag, residual=residual,
                         train=train)


def _stats_arena(cache, dev, dtype, shapes, route):
    """The BatchNorm partial-statistics buffers of a layer's forward.  The producing GEMM epilogues overwrite
    the same (row block, channel) entries on every call of one route and shape, and the entries they never
    write (rows past the kernel's row-block count, padded channels) must read as zero for bn_finalize — so a
    buffer kept per (device, dtype, shapes, route) in the layer's cache is zero-filled ONCE, not per forward.
    Streams: consumed by the layer's own bn_finalize right after, in stream order; the layer's next forward
    writes it again only after that.  Without a cache (bare calls): a fresh zeroed arena.  ``cache`` is the
    layer's sub-dict of this device (StgcnLayerFunction.forward), so eviction never touches another device's."""
    if cache is None:
        return K.zeros_arena(dev, *shapes)
    key = ("bn_stats", str(dev), dtype, tuple(map(tuple, shapes)), route)
    st = cache.get(key)
    if st is None:
        old = [k for k in list(cache) if isinstance(k, tuple) and k[:1] == ("bn_stats",)]
        for k in old[:-6]:  # keep a few shapes and routes (config 4 alternates 64- and 65-window units)
            del cache[k]
        st = cache[key] = K.zeros_arena(dev, *shapes)
    return st


@K.on_tensor_device
class StgcnLayerFunction(torch.autograd.Function):
    """Autograd node for the whole StgcnLayer (BN or LN variant)."""

    @staticmethod
    def forward(ctx, x, A, wg, bg, n1w, n1b, wt, bt, n2w, n2b, wr, br, nrw, nrb, cfg):
        kt, stride, residual, norm, dtype = cfg[:5]
        dev = x.device
        x = K.to_rows(x, dtype)
        N, Cin, T, V = x.shape
        P = A.shape[-3]
        Cout = wt.shape[0]
        pad = (kt - 1) // 2
        T_out = (T + 2 * pad - kt) // stride + 1
        M1, M2 = N * T * V, N * T_out * V
        A32 = A.detach().float().contiguous()
        res_conv = residual and not (Cin == Cout and stride == 1)
        packs = cfg[9] if len(cfg) > 9 else None  # LayerPacks of the model's PrepPlan launch, or None
        # the layer's cache, one sub-dict per device: DataParallel replicas share the module's dict (shallow
        # __dict__ copy) and run in one thread per device, so each thread only ever touches its own sub-dict
        # (dict.setdefault is atomic under the GIL)
        cache = cfg[8].setdefault(("dev", str(dev)), {}) if len(cfg) > 8 and cfg[8] is not None else None
        # SyncBatchNorm (syncbn.py): the statistics of every rank, else this rank's (the reference's DataParallel)
        sync = cfg[10] if len(cfg) > 10 else None
        bn_finalize = sync.finalize if sync is not None else K.bn_finalize

        # ---- graph convolution: g = sum_p A_p-mix(x) W_p + bias2d
        sup = cfg[5] if len(cfg) > 5 else None
        gather = sup is not None and A32.dim() == 3 and not sup.dense(P)
        if (gather and len(cfg) > 7 and cfg[7] and ROUTING.fused_inference and norm == LN
                and K.layer_fused_ok(sup, P, Cin, Cout, V, kt, stride, dtype)):
            # inference of a LayerNorm 64 -> 64 stride-1 layer: the one-kernel layer (g never leaves the chip;
            # nothing saved for backward): 0.12 vs 0.15-0.21 ms unfused
            return fused_layer_forward(x, A32, wg, bg, n1w, n1b, wt, bt, n2w, n2b, residual, dtype, cache=cache)
        if (gather and norm == LN and ROUTING.fused_ln_train and not (len(cfg) > 7 and cfg[7])
                and K.layer_fused_ok(sup, P, Cin, Cout, V, kt, stride, dtype)):
            # training forward of a LayerNorm 64 -> 64 stride-1 layer: the one-kernel layer (g and h on chip for
            # the temporal conv) also writes g, u and both LN statistics — exactly what the unfused forward
            # saves — so the backward below is unchanged (ln/ configs)
            y, g, u, ls1, ls2, h = fused_layer_forward(x, A32, wg, bg, n1w, n1b, wt, bt, n2w, n2b, residual, dtype,
                                                       cache=cache, train=True, packs=packs)
            ctx.cfg = cfg
            ctx.sup = sup
            ctx.dims = (N, Cin, Cout, T, T_out, V, P, pad, False)
            ctx.packs = None
            ctx.save_for_backward(x, A32, None, g, u, y, wg, bg, wt, n1w, n1b, n2w, n2b, ls1, ls2, h)
            ctx.in_dtype = A.dtype
            return y
        # gathered path: bias2d comes from the weight preparation below
        bias2d = None if gather else K.gcn_bias(A32, bg.detach().float().contiguous(), N, Cout)
        if norm == BN:  # all BatchNorm partial-statistics buffers of the layer from one zero fill
            cpo = -(-Cout // K.col_tile(Cout)) * K.col_tile(Cout)
            rb1 = K.gconv_row_blocks(N * T, V) if gather else K.row_blocks(M1, Cout)
            rb2 = K.row_blocks(M2, Cout)
            st_shapes = [(rb1, cpo, 4), (rb2, cpo, 4)] + ([(K.row_blocks(M2, Cout), cpo, 4)] if res_conv else [])
            st_all = _stats_arena(cache, dev, x.dtype, st_shapes, gather)
            st1, st2 = st_all[0], st_all[1]
            str_ = st_all[2] if res_conv else None
        # ---- residual branch: independent of the graph conv -> temporal conv chain until the output norm
        r = None
        if res_conv:
            wrp, cpr, kpr = packs.wr if packs is not None else \
                K.pack_weight(wr.detach().float().view(1, Cout, Cin), dtype)
            r = K.conv_rows(x, wrp, Cin, Cout, cpr, kpr, T, T_out, Kt=1, stride=stride, pad=0,
                            bias=br.detach().float().contiguous(), stats=str_ if norm == BN else None)
            if norm == BN:
                mrr, scr, shr = bn_finalize(str_, str_.shape[0], cpr, Cout, nrw.detach().float(), nrb.detach().float())
            else:
                lsr = K.ln_stats(r, N * T_out, V, Cout)

        if gather:  # joint-gathered GEMM over per-joint effective weights (gconv.hip), no XA in HBM
            if packs is not None and packs.gw is not None:
                wgp, bias2d = packs.gw
            else:
                wg2 = wg.detach().float().reshape(P * Cout, Cin).contiguous()
                wgp, bias2d = K.gconv_weights(A32, wg2, sup, Cout, Cin, False, dtype,
                                              bias=bg.detach().float().contiguous())
            cpg, kpg = wgp.shape[2], wgp.shape[3]
            if norm == BN:
                assert cpg == cpo
            g = K.gconv(x, wgp, sup, Cin, Cout, bias=bias2d, stats=st1 if norm == BN else None)
            XA = None
        else:
            XA = K.amix_fwd(x, A32)
            wg3 = wg.detach().float().view(P, Cout, Cin).permute(1, 0, 2).reshape(1, Cout, P * Cin)
            wgp, cpg, kpg = K.pack_weight(wg3, dtype)
            bmode = 3 if A32.dim() == 4 else 2
            g = K.conv_rows(XA, wgp, P * Cin, Cout, cpg, kpg, T, T, bias=bias2d, bias_mode=bmode,
                            stats=st1 if norm == BN else None)
        if norm == BN:
            mr1, sc1, sh1 = bn_finalize(st1, st1.shape[0], cpg, Cout, n1w.detach().float(), n1b.detach().float())
            pro1 = dict(pro=1, pro_a=sc1, pro_b=sh1)
        else:
            # LayerNorm: h = relu(LN1(g)) is materialised (one HBM-bound pass, ln.hip) and the temporal conv runs
            # without a prologue on the persistent kernels; a per-frame-statistics, per-(c,v)-affine prologue
            # in the conv tiles measured 304 us vs ~85 us for this pass + conv_wide at 64 -> 64.  h is kept for
            # the weight gradient.
            ls1 = K.ln_stats(g, N * T, V, Cout)
            h = K.ln_apply(g, ls1, _flat_ln(n1w), _flat_ln(n1b), M1, V, Cout, relu=True)
            pro1 = {}

        # ---- temporal conv on relu(norm1(g)) (norm applied in the prologue)
        wtp, cpt, kpt = packs.wt if packs is not None else \
            K.pack_weight(wt.detach().float().squeeze(-1).permute(2, 0, 1), dtype, stride=stride)  # [Kt][Cout][Cin]
        u = K.conv_rows(g if norm == BN else h, wtp, Cout, Cout, cpt, kpt, T, T_out, Kt=kt, stride=stride,
                        pad=pad, bias=bt.detach().float().contiguous(), stats=st2 if norm == BN else None,
                        tag=f"tcn_fwd_c{Cout}" if stride == 1 else None, **pro1)

        # ---- y = relu(norm2(u) + res)
        if norm == BN:
            mr2, sc2, sh2 = bn_finalize(st2, st2.shape[0], cpt, Cout, n2w.detach().float(), n2b.detach().float())
            # the output's sign bits for the backward's ReLU mask (the fused BN backward reads them instead of y:
            # 1/16 of the bytes in both of its passes)
            ybits = torch.empty((M2, Cout // 8), dtype=torch.uint8, device=dev) \
                if (ROUTING.bn_mask_bits and dtype == torch.bfloat16 and K.bn_fused_ok(Cout, dtype) and Cout % 8 == 0) \
                else None
            if res_conv:
                y = K.bn_apply(u, sc2, sh2, M2, Cout, res_mode=2, r=r, rsc=scr, rsh=shr, bits=ybits)
            else:
                y = K.bn_apply(u, sc2, sh2, M2, Cout, res_mode=1 if residual else 0, r=x if residual else None,
                               bits=ybits)
        else:
            ls2 = K.ln_stats(u, N * T_out, V, Cout)
            g2, b2 = _flat_ln(n2w), _flat_ln(n2b)
            if res_conv:
                y = K.ln_apply(u, ls2, g2, b2, M2, V, Cout, res_mode=2, r=r, rst=lsr, rg=_flat_ln(nrw),
                               rb=_flat_ln(nrb))
            else:
                y = K.ln_apply(u, ls2, g2, b2, M2, V, Cout, res_mode=1 if residual else 0,
                               r=x if residual else None)

        ctx.cfg = cfg
        ctx.sup = sup if gather else None
        ctx.dims = (N, Cin, Cout, T, T_out, V, P, pad, res_conv)
        ctx.packs = (cpg, kpg, cpt, kpt)
        saved = [x, A32, XA, g, u, y, wg, bg, wt, n1w, n1b, n2w, n2b]
        if norm == BN:
            saved += [mr1, sc1, sh1, mr2, ybits]
        else:
            saved += [ls1, ls2, h]
        if res_conv:
            saved += [r, wr, nrw, nrb] + ([mrr] if norm == BN else [lsr])
        ctx.save_for_backward(*saved)
        ctx.in_dtype = A.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        kt, stride, residual, norm, dtype = ctx.cfg[:5]
        N, Cin, Cout, T, T_out, V, P, pad, res_conv = ctx.dims
        sv = list(ctx.saved_tensors)
        x, A32, XA, g, u, y, wg, bg, wt, n1w, n1b, n2w, n2b = sv[:13]
        rest = sv[13:]
        ybits = None
        if norm == BN:
            mr1, sc1, sh1, mr2, ybits = rest[:5]
            rest = rest[5:]
        else:
            ls1, ls2, h = rest[:3]
            rest = rest[3:]
        if res_conv:
            r, wr, nrw, nrb, strr = rest
        dev = x.device
        dy = K.to_rows(dy, dtype)
        M1, M2 = N * T * V, N * T_out * V
        packs = ctx.cfg[9] if len(ctx.cfg) > 9 else None
        sync = ctx.cfg[10] if len(ctx.cfg) > 10 else None
        grads = {}
        # the temporal / residual weight gradients come back in nn.Conv2d order, overwritten (conv_wgrad_w); the
        # graph-conv accumulation targets (dW, dA, per-joint row sums) are zero-filled only on the routes that
        # accumulate into them (one fill for all three)
        zl = {}

        def zero_targets():
            if not zl:
                zl["t"] = K.zeros_arena(dev, (P * Cout, Cin), (P, V, V),
                                        (N, V, Cout) if A32.dim() == 4 else (V, Cout))
            return zl["t"]

        # ---- through relu(norm2(u) + res): dz = dy * [y > 0]
        du = K.cl_empty(N, Cout, T_out, V, dtype, dev)
        dx = K.cl_empty(N, Cin, T, V, dtype, dev)
        dx_written = False
        fused = norm == BN and K.bn_fused_ok(Cout, dtype)
        # identity residual with the forward's sign bits and the gathered graph conv: its masked gradient
        # dy * [y > 0] is added in the graph conv's data-gradient epilogue (not written to dx by the BN backward)
        res_in_gconv = fused and residual and not res_conv and ybits is not None and ctx.sup is not None
        bt_done = False
        if fused:
            # one reduce + one apply pass: du, the residual branch's dr (or dx = dz), and the conv-bias
            # gradients (column sums of du / dr) together
            kw = dict(mask=1, mref=y, x1=u, mr1=mr2, g1=n2w.detach().float(), out1=du, bias_sums=True)
            if ybits is not None:
                kw.update(mask=3, mref=ybits)
            if res_conv:
                dr = K.cl_empty(N, Cout, T_out, V, dtype, dev)
                kw.update(x2=r, mr2=strr, g2=nrw.detach().float(), out2=dr)
            elif residual and not res_in_gconv:
                kw.update(out2=dx)
                dx_written = True
            sums2, osum2 = K.bn_bwd_fused(dy, M2, Cout, sync=sync, **kw)
            grads["n2w"], grads["n2b"] = sums2[1], sums2[0]
            grads["bt"] = osum2[0]
            bt_done = True
            if res_conv:  # nrb == n2b numerically; own storage so no two parameters share a grad tensor
                grads["nrw"], grads["nrb"] = sums2[2], sums2[0].clone()
                grads["br"] = osum2[1]
        elif norm == BN:
            s2 = K.bn_bwd_reduce(dy, M2, Cout, mask=1, mref=y, x=u, mean_rstd=mr2)
            grads["n2w"], grads["n2b"] = s2[:, 1].clone(), s2[:, 0].clone()
            if sync is not None:
                sync.all_reduce_sums(s2, M2)
            K.bn_bwd_apply(dy, M2, Cout, du, mask=1, mref=y, x=u, mean_rstd=mr2, gamma=n2w.detach().float(), sums=s2)
        else:
            dgb2 = torch.zeros((2, Cout * V), dtype=torch.float32, device=dev)
            K.ln_bwd(dy, u, ls2, _flat_ln(n2w), _flat_ln(n2b), N * T_out, V, Cout, du, mask=1, mref=y, dgb=dgb2)
            grads["n2w"], grads["n2b"] = dgb2[0].view(n2w.shape), dgb2[1].view(n2b.shape)

        if res_conv:
            if not fused:
                dr = K.cl_empty(N, Cout, T_out, V, dtype, dev)
                if norm == BN:
                    sr = K.bn_bwd_reduce(dy, M2, Cout, mask=1, mref=y, x=r, mean_rstd=strr)
                    grads["nrw"], grads["nrb"] = sr[:, 1].clone(), sr[:, 0].clone()
                    if sync is not None:
                        sync.all_reduce_sums(sr, M2)
                    K.bn_bwd_apply(dy, M2, Cout, dr, mask=1, mref=y, x=r, mean_rstd=strr,
                                   gamma=nrw.detach().float(), sums=sr)
                else:
                    dgbr = torch.zeros((2, Cout * V), dtype=torch.float32, device=dev)
                    K.ln_bwd(dy, r, strr, _flat_ln(nrw), _flat_ln(nrb), N * T_out, V, Cout, dr, mask=1, mref=y,
                             dgb=dgbr)
                    grads["nrw"], grads["nrb"] = dgbr[0].view(nrw.shape), dgbr[1].view(nrb.shape)
                grads["br"] = K.bn_bwd_reduce(dr, M2, Cout)[:, 0].clone()
            # residual conv (1x1, stride s, bias): data grad (transposed), weight grad
            wrTp, cq, kq = packs.wrT if packs is not None else \
                K.pack_weight(wr.detach().float().view(Cout, Cin).t().unsqueeze(0), dtype)
            grads["wr"] = K.conv_wgrad_w(x, dr, Cin, Cout, T, T_out, Kt=1, stride=stride, pad=0).view(Cout, Cin, 1, 1)
            K.conv_rows(dr, wrTp, Cout, Cin, cq, kq, T_out, T, Kt=1, stride=stride, pad=0, trans=True, out=dx)
            dx_written = True
        elif residual and not fused:
            K.bn_bwd_apply(dy, M2, Cin, dx, mask=1, mref=y)  # dx = dz
            dx_written = True

        # ---- temporal conv: dh = conv^T(du), dWt, dbt
        # [Kt][Cin=Cout][Cout]: W[co][ci][dt] -> [dt][ci][co]
        wtTp, cq, kq = packs.wtT if packs is not None else \
            K.pack_weight(wt.detach().float().squeeze(-1).permute(2, 1, 0), dtype, stride=stride, trans=True)
        if norm == BN:
            pro1, hin = dict(pro=1, pro_a=sc1, pro_b=sh1), g
        else:  # the forward's h = relu(LN1(g)), recomputed when the forward did not keep it (fused route)
            pro1 = {}
            hin = h if h is not None else K.ln_apply(g, ls1, _flat_ln(n1w), _flat_ln(n1b), M1, V, Cout, relu=True)
        grads["wt"] = K.conv_wgrad_w(hin, du, Cout, Cout, T, T_out, Kt=kt, stride=stride, pad=pad,
                                     **pro1).unsqueeze(-1)  # (co, ci, Kt, 1)
        if K.tconv_frame_ok(Cout, kt, stride, V, dtype) and getattr(wtTp, "frag_stride", None) == 1:
            dh = K.tconv_frame(du, wtTp, cq, kq, trans=True)
        else:
            dh = K.conv_rows(du, wtTp, Cout, Cout, cq, kq, T_out, T, Kt=kt, stride=stride, pad=pad, trans=True)
        if not bt_done:
            grads["bt"] = K.bn_bwd_reduce(du, M2, Cout)[:, 0].clone()

        # ---- through relu(norm1(g))
        dg = K.cl_empty(N, Cout, T, V, dtype, dev)
        if fused:
            s1, _ = K.bn_bwd_fused(dh, M1, Cout, mask=2, mref=g, msc=sc1, msh=sh1, x1=g, mr1=mr1,
                                   g1=n1w.detach().float(), out1=dg, sync=sync)
            grads["n1w"], grads["n1b"] = s1[1], s1[0]
        elif norm == BN:
            s1 = K.bn_bwd_reduce(dh, M1, Cout, mask=2, mref=g, msc=sc1, msh=sh1, x=g, mean_rstd=mr1)
            grads["n1w"], grads["n1b"] = s1[:, 1].clone(), s1[:, 0].clone()
            if sync is not None:
                sync.all_reduce_sums(s1, M1)
            K.bn_bwd_apply(dh, M1, Cout, dg, mask=2, mref=g, msc=sc1, msh=sh1, x=g, mean_rstd=mr1,
                           gamma=n1w.detach().float(), sums=s1)
        else:
            dgb1 = torch.zeros((2, Cout * V), dtype=torch.float32, device=dev)
            K.ln_bwd(dh, g, ls1, _flat_ln(n1w), _flat_ln(n1b), N * T, V, Cout, dg, mask=2, dgb=dgb1)
            grads["n1w"], grads["n1b"] = dgb1[0].view(n1w.shape), dgb1[1].view(n1b.shape)

        # ---- graph convolution backward
        bgp = bg.detach().float().view(P, Cout)
        if ctx.sup is not None:
            # data grad: same gather GEMM on dg over the reverse lists with transposed effective weights;
            # weight / adjacency / bias grads through the per-joint dWeff[w][j] = sum_i dg[(i,w)] x[(i,S(w)_j)]^T blocks
            sup = ctx.sup
            wg2 = wg.detach().float().reshape(P * Cout, Cin).contiguous()
            _gconv_wgrad_dweff(ctx, x, dg, A32, wg, wg2, bg, bgp, sup, grads, zero_targets, P, Cin, Cout, T, V, M1,
                               dtype, dev)
            dA = grads.pop("dA")
            wgT = packs.gwT if packs is not None and packs.gwT is not None else \
                K.gconv_weights(A32, wg2, sup, Cout, Cin, True, dtype)
            K.gconv(dg, wgT, sup, Cout, Cin, trans=True, out=dx, accumulate=dx_written,
                    res=(dy, ybits) if res_in_gconv else None)
        else:
            # DW[(n,t,w)][p*Cin+ci] = sum_c dg[(n,t,w)][c] Wg[p*Cout+c][ci]
            wgT = wg.detach().float().view(P, Cout, Cin).permute(0, 2, 1).reshape(1, P * Cin, Cout)
            wgTp, cq, kq = K.pack_weight(wgT, dtype)
            DW = K.conv_rows(dg, wgTp, Cout, P * Cin, cq, kq, T, T)
            K.amix_trans(DW, A32, Cin, dx, accumulate=dx_written)
            dA = K.amix_dA(x, DW, A32)
            dwg = K.conv_wgrad(XA, dg, P * Cin, Cout, T, T, Kt=1)              # [1][Cout][P*Cin]
            grads["wg"] = dwg.view(Cout, P, Cin).permute(1, 0, 2).reshape(P * Cout, Cin, 1, 1)
            dA = _bias_through_A(dA, A32, bg, bgp, dg, None, zero_targets()[2], M1, Cout, V, grads)

        def gr(name, like):
            v = grads.get(name)
            if v is None or like is None or not like.requires_grad:
                return None
            return v.to(like.dtype).view(like.shape)

        wr_, br_, nrw_, nrb_ = (wr, None, nrw, nrb) if res_conv else (None, None, None, None)
        return (dx, dA.to(ctx.in_dtype), gr("wg", wg), gr("bg", bg), gr("n1w", n1w), gr("n1b", n1b), gr("wt", wt),
                grads["bt"], gr("n2w", n2w), gr("n2b", n2b), gr("wr", wr_),
                grads.get("br"), gr("nrw", nrw_), gr("nrb", nrb_), None)


def _bias_through_A(dA, A32, bg, bgp, dg, S_fused, z_S, M1, Cout, V, grads):
    """Bias pushed through A: dA[p][v][w] += sum_c b_p[c] S[w][c] (independent of v), S = per-joint row
    sums of dg (already produced by the joint-grouped weight-gradient kernel when S_fused is given);
    sets grads["bg"] and returns dA."""
    if A32.dim() == 4:
        Sn = K.rowgroup_sum(dg, M1, Cout, V, per_sample=True, out=z_S)   # [N][V(w)][Cout]
        dA = dA + torch.einsum("pc,nwc->npw", bgp, Sn).unsqueeze(2)
        colsum = A32.sum(dim=2)                                         # [N][P][W]
        grads["bg"] = torch.einsum("npw,nwc->pc", colsum, Sn).reshape(-1)
        return dA
    S = S_fused if S_fused is not None else K.rowgroup_sum(dg, M1, Cout, V, out=z_S)   # [V(w)][Cout]
    if not dA.is_contiguous():
        dA = dA.contiguous()
    grads["bg"] = K.gcn_bias_bwd(A32, bg.detach().float().contiguous(), S, dA, Cout)
    return dA


def _gconv_wgrad_dweff(ctx, x, dg, A32, wg, wg2, bg, bgp, sup, grads, zero_targets, P, Cin, Cout, T, V, M1, dtype,
                       dev):
    """Graph-conv weight / adjacency / bias gradients through the per-joint dWeff[w][j] = sum_i dg[(i,w)]
    x[(i,S(w)_j)]^T blocks (gconv_wgrad + finish).
    Sets grads["wg"], grads["bg"], grads["dA"]."""
    fuse_s = A32.dim() == 3 and K.gconv_wgrad_rowsum_ok(sup, Cin, Cout, dtype)
    dense_dA = ctx.cfg[6] and ctx.needs_input_grad[1]
    # row sums: overwritten by the joint-grouped wgrad kernel
    S_rows = torch.empty((V, Cout), dtype=torch.float32, device=dev) if fuse_s else None
    dweff = K.gconv_wgrad(x, dg, sup, Cin, Cout, rowsum=S_rows)
    if fuse_s and not dense_dA and K.gconv_finish_bias_ok(A32, sup):
        # dW, dA (support + bias through A) and db in two launches, outputs overwritten
        dwg2, dA, grads["bg"] = K.gconv_finish_bias(dweff, A32, wg2, sup, Cout, Cin, bg.detach().float().contiguous(),
                                                    S_rows)
        dA_done = True
    else:
        z_dwg, z_dA, z_S = zero_targets()
        dwg2, dA = K.gconv_finish(dweff, A32, wg2, sup, Cout, Cin, dW=z_dwg, dA=z_dA)
        dA_done = False
    grads["wg"] = dwg2.view(P * Cout, Cin, 1, 1)
    if dense_dA:
        # caller-owned A: the reference's dA is dense (also off the graph's support), so take
        # it from the A-first factorisation dA_p[v][w] = sum x[(i,v)] . (dg W_p)[(i,w)]
        wgTd = wg.detach().float().view(P, Cout, Cin).permute(0, 2, 1).reshape(1, P * Cin, Cout)
        wgTp, cq, kq = K.pack_weight(wgTd, dtype)
        dA = K.amix_dA(x, K.conv_rows(dg, wgTp, Cout, P * Cin, cq, kq, T, T), A32)
    if not dA_done:
        dA = _bias_through_A(dA, A32, bg, bgp, dg, S_rows, zero_targets()[2], M1, Cout, V, grads)
    grads["dA"] = dA


@K.on_tensor_device
class GcnFunction(torch.autograd.Function):
    """ConvTemporalGraphical.forward alone (models/utils/tgcn.py:58-79): conv1x1(+bias) -> @A -> sum_P."""

    @staticmethod
    def forward(ctx, x, A, wg, bg, dtype):
        x = K.to_rows(x, dtype)
        N, Cin, T, V = x.shape
        P = A.shape[-3]
        Cout = wg.shape[0] // P
        A32 = A.detach().float().contiguous()
        XA = K.amix_fwd(x, A32)
        wg3 = wg.detach().float().view(P, Cout, Cin).permute(1, 0, 2).reshape(1, Cout, P * Cin)
        wgp, cp, kp = K.pack_weight(wg3, dtype)
        bias2d = K.gcn_bias(A32, bg.detach().float().contiguous(), N, Cout)
        g = K.conv_rows(XA, wgp, P * Cin, Cout, cp, kp, T, T, bias=bias2d, bias_mode=3 if A32.dim() == 4 else 2)
        ctx.save_for_backward(x, A32, XA, wg, bg)
        ctx.meta = (dtype, A.dtype)
        return g

    @staticmethod
    def backward(ctx, dg):
        x, A32, XA, wg, bg = ctx.saved_tensors
        dtype, adt = ctx.meta
        N, Cin, T, V = x.shape
        P = A32.shape[-3]
        Cout = wg.shape[0] // P
        dg = K.to_rows(dg, dtype)
        M = N * T * V
        wgT = wg.detach().float().view(P, Cout, Cin).permute(0, 2, 1).reshape(1, P * Cin, Cout)
        wgTp, cq, kq = K.pack_weight(wgT, dtype)
        DW = K.conv_rows(dg, wgTp, Cout, P * Cin, cq, kq, T, T)
        dx = K.cl_empty(N, Cin, T, V, dtype, x.device)
        K.amix_trans(DW, A32, Cin, dx, accumulate=False)
        dA = K.amix_dA(x, DW, A32)
        bgp = bg.detach().float().view(P, Cout)
        if A32.dim() == 4:
            Sn = K.rowgroup_sum(dg, M, Cout, V, per_sample=True)
            dA += torch.einsum("pc,nwc->npw", bgp, Sn).unsqueeze(2)
            dbg = torch.einsum("npw,nwc->pc", A32.sum(dim=2), Sn).reshape(-1)
        else:
            S = K.rowgroup_sum(dg, M, Cout, V)
            dA += (bgp @ S.t()).unsqueeze(1)
            dbg = (A32.sum(dim=1) @ S).reshape(-1)
        dwg = K.conv_wgrad(XA, dg, P * Cin, Cout, T, T, Kt=1)
        dwg = dwg.view(Cout, P, Cin).permute(1, 0, 2).reshape(P * Cout, Cin, 1, 1)
        return dx, dA.to(adt), dwg.to(wg.dtype), dbg.to(bg.dtype), None


def plan_conv1x1_packs(plan, w, dtype):
    """Forward and data-gradient packs of a 1x1 conv weight (Cout, Cin', 1, 1) for Conv1x1Function; Cin' may
    be below the activation's channel count (fcn_in: 3 input features in 8-channel rows), the packs pad."""
    Cout, Ci = w.shape[0], w.shape[1]
    w2 = w.detach().view(Cout, Ci)
    return K.pack_weight(w2.unsqueeze(0), dtype, plan=plan), K.pack_weight(w2.t().unsqueeze(0), dtype, plan=plan)


@K.on_tensor_device
class Conv1x1Function(torch.autograd.Function):
    """Pointwise conv on channels-last rows (fcn_in / fcn_out, stgcn.py:49,74): y = W x + b.  w may have fewer
    input channels than x (fcn_in's 3 features in 8-channel rows: the missing columns act as zeros); packs =
    plan_conv1x1_packs(...) filled by the model's PrepPlan launch, or None (packed here)."""

    @staticmethod
    def forward(ctx, x, w, b, dtype, packs=None):
        x = K.to_rows(x, dtype)
        N, Cin, T, V = x.shape
        Cout, Ci = w.shape[0], w.shape[1]
        wp, cp, kp = packs[0] if packs is not None else \
            K.pack_weight(w.detach().float().view(Cout, Ci).unsqueeze(0), dtype)
        y = K.conv_rows(x, wp, Cin, Cout, cp, kp, T, T, bias=b.detach().float().contiguous())
        ctx.save_for_backward(x, w)
        ctx.dtype = dtype
        ctx.packT = packs[1] if packs is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dtype = ctx.dtype
        N, Cin, T, V = x.shape
        Cout, Ci = w.shape[0], w.shape[1]
        dy = K.to_rows(dy, dtype)
        wT, cq, kq = ctx.packT if ctx.packT is not None else \
            K.pack_weight(w.detach().float().view(Cout, Ci).t().unsqueeze(0), dtype)
        dx = K.conv_rows(dy, wT, Cout, Cin, cq, kq, T, T, trans=True)
        dw = K.conv_wgrad_w(x, dy, Cin, Cout, T, T).view(Cout, Cin, 1, 1)
        if Ci < Cin:
            dw = dw[:, :Ci]
        db = K.bn_bwd_reduce(dy, N * T * V, Cout)[:, 0]
        return dx, dw.to(w.dtype), db.to(w.dtype), None, None


@K.on_tensor_device
class InputBatchNormFunction(torch.autograd.Function):
    """BatchNorm1d(V*C) on (N, V*C, T) (models/utils/batchnorm.py:13-23): per-(v,c) batch stats over
    (N,T).  Channels-last NTVC rows are exactly [N*T][V*C], so it is a row BatchNorm with V*C channels."""

    @staticmethod
    def forward(ctx, x, w, b, dtype, sync=None):
        x = K.to_rows(x, dtype)
        N, C, T, V = x.shape
        if K.rows_ld(x) != C:
            x = x.contiguous(memory_format=torch.channels_last)
        F_, CV = N * T, V * C
        part, nb, _ = K.bn_stats_partial(x, F_, CV, ld=CV)
        # reference weight index = v*C + c == channels-last (v, c) order
        mr, sc, sh = (sync.finalize if sync is not None else K.bn_finalize)(part, nb, CV, CV, w.detach().float(),
                                                                            b.detach().float())
        y = K.cl_empty(N, C, T, V, dtype, x.device)
        K.bn_apply(x, sc, sh, F_, CV, relu=False, out=y, ldu=CV, ldy=CV)
        ctx.save_for_backward(x, w, mr)
        ctx.dtype = dtype
        ctx.sync = sync
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mr = ctx.saved_tensors
        N, C, T, V = x.shape
        F_, CV = N * T, V * C
        dy = K.to_rows(dy, ctx.dtype)
        if K.rows_ld(dy) != C:
            dy = dy.contiguous(memory_format=torch.channels_last)
        sums = _bn_reduce_flat(dy, x, mr, F_, CV)
        dw, db = sums[:, 1].to(w.dtype), sums[:, 0].to(w.dtype)
        if ctx.sync is not None:  # the parameter gradients keep this rank's own sums (copies: sums is exchanged)
            dw, db = dw.clone(), db.clone()
            ctx.sync.all_reduce_sums(sums, F_)
        dx = K.cl_empty(N, C, T, V, ctx.dtype, x.device)
        _bn_apply_flat(dy, x, mr, w.detach().float(), sums, F_, CV, dx)
        return dx, dw, db, None, None


@K.on_tensor_device
class WindowStageFunction(torch.autograd.Function):
    """norm_in + fcn_in of a batch of sliding windows (WindowSegment, segment_generator.py:132-145; stgcn.py:
    82-85) straight from the padded capture (1, Cin, Lp, V): windows [n0, n0+nw) of W frames, never formed
    (window.hip).  mode 0: BatchNorm1d(V*Cin) with the windowed batch's statistics (each frame weighted by
    the windows holding it); mode 1: the per-frame LayerNorm([Cin,1,V]).  Returns the first activation
    (nw, Cout, W, V) channels-last; backward gives the norm and fcn_in parameter gradients (the capture
    takes none, as in the reference where it is data)."""

    @staticmethod
    def forward(ctx, capture, n0, nw, W, norm_w, norm_b, w, b, mode, dtype, sync=None):
        Cout = w.shape[0]
        w2 = w.detach().float().reshape(Cout, -1)
        bias = b.detach().float() if b is not None else None
        g, be = norm_w.detach().float().reshape(-1), norm_b.detach().float().reshape(-1)
        if mode == 0:
            part, nb = K.window_stats(capture, W, n0, nw, 0)
            VC = part.shape[1]
            # SyncBatchNorm: only the forward statistics are exchanged (the capture takes no gradient, and the
            # parameter gradients are this rank's own sums)
            st, sc, sh = (sync.finalize if sync is not None else K.bn_finalize)(part, nb, VC, VC, g, be)
            y = K.window_expand(capture, W, n0, nw, 0, sc, sh, None, w2, bias, dtype)
        else:
            st, _ = K.window_stats(capture, W, n0, nw, 1)
            y = K.window_expand(capture, W, n0, nw, 1, g, be, st, w2, bias, dtype)
        ctx.save_for_backward(capture, norm_w, norm_b, w, b, st)
        ctx.cfg = (n0, nw, W, mode)
        return y

    @staticmethod
    def backward(ctx, dy):
        capture, norm_w, norm_b, w, b, st = ctx.saved_tensors
        n0, nw, W, mode = ctx.cfg
        dy = K.to_rows(dy, dy.dtype)
        Cout = w.shape[0]
        dg, dbe, dw, db = K.window_grad(dy, capture, W, n0, nw, mode, st, norm_w.detach().float().reshape(-1),
                                        norm_b.detach().float().reshape(-1), w.detach().float().reshape(Cout, -1))
        return (None, None, None, None, dg.view(norm_w.shape).to(norm_w.dtype), dbe.view(norm_b.shape).to(norm_b.dtype),
                dw.view(w.shape).to(w.dtype), None if b is None else db.to(b.dtype), None, None, None)


def stage_window_batch(xb, norm_in, fcn_in, dtype):
    """norm_in (modules.BatchNorm1d or LayerNorm) + fcn_in of a segment.WindowBatch, from its capture."""
    ln = not hasattr(norm_in, "norm")  # modules.BatchNorm1d wraps nn.BatchNorm1d as .norm
    g, b = (norm_in.weight, norm_in.bias) if ln else (norm_in.norm.weight, norm_in.norm.bias)
    return WindowStageFunction.apply(xb.capture, xb.n0, xb.nw, xb.W, g, b, fcn_in.weight, fcn_in.bias,
                                     1 if ln else 0, dtype, None if ln else active_sync(norm_in))


def _as_rows(t, F_, CV):
    # a (F_, 1, 1, CV) contiguous buffer viewed as logical (F_, CV, 1, 1) channels-last
    return t.permute(0, 2, 3, 1).contiguous().view(F_, 1, 1, CV).permute(0, 3, 1, 2)


def _bn_reduce_flat(dy, x, mr, F_, CV):
    return K.bn_bwd_reduce(_as_rows(dy, F_, CV), F_, CV, x=_as_rows(x, F_, CV), mean_rstd=mr)


def _bn_apply_flat(dy, x, mr, gamma, sums, F_, CV, dx):
    out = _as_rows(dx, F_, CV)
    K.bn_bwd_apply(_as_rows(dy, F_, CV), F_, CV, out, x=_as_rows(x, F_, CV), mean_rstd=mr, gamma=gamma, sums=sums)
    return out


@K.on_tensor_device
class LayerNormFunction(torch.autograd.Function):
    """Custom LayerNorm([C,1,V]) (models/utils/layernorm.py:22-28) on channels-last rows."""

    @staticmethod
    def forward(ctx, x, w, b, dtype):
        x = K.to_rows(x, dtype)
        N, C, T, V = x.shape
        st = K.ln_stats(x, N * T, V, C)
        y = K.ln_apply(x, st, _flat_ln(w), _flat_ln(b), N * T * V, V, C, relu=False)
        ctx.save_for_backward(x, w, b, st)
        ctx.dtype = dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, st = ctx.saved_tensors
        N, C, T, V = x.shape
        dy = K.to_rows(dy, ctx.dtype)
        dx = K.cl_empty(N, C, T, V, ctx.dtype, x.device)
        dgb = torch.zeros((2, C * V), dtype=torch.float32, device=x.device)
        K.ln_bwd(dy, x, st, _flat_ln(w), _flat_ln(b), N * T, V, C, dx, dgb=dgb)
        return dx, dgb[0].view(w.shape).to(w.dtype), dgb[1].view(b.shape).to(b.dtype), None


@K.on_tensor_device
class PoolFunction(torch.autograd.Function):
    """F.avg_pool2d(x, x.size()[2:]) (stgcn.py:92) -> (N, C, 1, 1); joints_only=True is the RT head's
    AvgPool2d((1, V)) (rtstgcn.py:127,149) -> (N, C, T, 1)."""

    @staticmethod
    def forward(ctx, x, dtype, joints_only=False):
        x = K.to_rows(x, dtype)
        N, C, T, V = x.shape
        ctx.shape = (N, C, T, V)
        ctx.dtype = dtype
        ctx.joints_only = joints_only
        if joints_only:
            return K.pool_rows(x, N * T, V, C).reshape(N, T, 1, C).permute(0, 3, 1, 2)
        return K.pool_rows(x, N, T * V, C)

    @staticmethod
    def backward(ctx, dp):
        N, C, T, V = ctx.shape
        dp = K.to_rows(dp, ctx.dtype)
        dx = K.cl_empty(N, C, T, V, ctx.dtype, dp.device)
        if ctx.joints_only:
            dp = dp.permute(0, 2, 3, 1).reshape(N * T, 1, 1, C).permute(0, 3, 1, 2)
            K.unpool_rows(dp, V, C, N * T * V, dx)
        else:
            K.unpool_rows(dp, T * V, C, N * T * V, dx)
        return dx, None, None


def _strided_rows_ok(t, dtype) -> bool:
    """A (N, C, T, V) tensor the row kernels can read in place: the dtype, unit channel stride and evenly
    strided rows (K.rows_ld)."""
    if t.dtype != dtype or t.dim() != 4 or t.stride(1) != 1 or not t.is_cuda:
        return False
    try:
        K.rows_ld(t)
    except RuntimeError:
        return False
    return True


@K.on_tensor_device
class AttentionFunction(torch.autograd.Function):
    """C = softmax(theta^T phi) per (n, p) (models/aagcn/aagcn.py:142-145), theta/phi channels-last rows."""

    @staticmethod
    def forward(ctx, theta, phi, P, dtype):
        # strided rows are fine (the kernels take a row stride): attn_proj's theta / phi are the two channel
        # halves of one row buffer, and keeping them there lets attn_bwd return both gradients in one buffer
        theta = theta if _strided_rows_ok(theta, dtype) else K.to_rows(theta, dtype)
        phi = phi if _strided_rows_ok(phi, dtype) else K.to_rows(phi, dtype)
        C = K.attn_scores(theta, phi, P)
        ctx.save_for_backward(theta, phi, C)
        ctx.P = P
        ctx.dtype = dtype
        return C

    @staticmethod
    def backward(ctx, dC):
        theta, phi, C = ctx.saved_tensors
        dth, dph = K.attn_bwd(theta, phi, ctx.P, C, dC.float().contiguous())
        return dth, dph, None, None


def attn_proj_ok(x, Cin, Nt, Np, dtype) -> bool:
    return dtype == torch.bfloat16 and Cin % 16 == 0 and Cin <= 256 and Nt % 4 == 0 and Np % 4 == 0


@K.on_tensor_device
class AttnProjFunction(torch.autograd.Function):
    """AgcnLayer's theta and phi 1x1 convs (aagcn.py:139-141) for a bf16 model: one fp32-output projection
    of the bf16 activation (stgcn_attn_proj: no fp32 copy of x, no fp32 GEMM), theta and phi the two
    channel halves of one row buffer.  Backward: the two gradients (one buffer from attn_bwd) rounded to
    bf16 once, then the bf16 transposed 1x1 conv (dx) and weight-gradient kernels; the bias gradients are
    column sums of the fp32 gradients."""

    @staticmethod
    def forward(ctx, x, wt, bt, wp, bp):
        x = K.to_rows(x, torch.bfloat16)
        Nt, Np = wt.shape[0], wp.shape[0]
        Cin = x.shape[1]
        W = torch.cat([wt.detach().float().reshape(Nt, Cin), wp.detach().float().reshape(Np, Cin)])
        b = torch.cat([bt.detach().float(), bp.detach().float()])
        out = K.attn_proj(x, W, b)
        ctx.save_for_backward(x, W)
        ctx.split = (Nt, Np)
        ctx.shapes = (wt.shape, wp.shape, wt.dtype)
        return out[:, :Nt], out[:, Nt:]

    @staticmethod
    def backward(ctx, dth, dph):
        x, W = ctx.saved_tensors
        Nt, Np = ctx.split
        N, Cin, T, V = x.shape
        Nout = Nt + Np
        es = dth.element_size()
        if (dth.dim() == 4 and K.rows_ld(dth) == Nout and K.rows_ld(dph) == Nout
                and dph.data_ptr() - dth.data_ptr() == Nt * es):
            D = torch.as_strided(dth, (N, Nout, T, V), dth.stride())  # the attn_bwd buffer, both halves
        else:
            D = torch.cat([dth, dph], 1).contiguous(memory_format=torch.channels_last)
        D = D.float()
        # the bf16 GEMM operand and the bias gradients (column sums of the fp32 values) from one read of D
        D16, db = K.cast_colsum(D, N * T * V, Nout)
        wT, cq, kq = K.pack_weight(W.t().reshape(1, Cin, Nout), torch.bfloat16)
        dx = K.conv_rows(D16, wT, Nout, Cin, cq, kq, T, T, trans=True)
        dW = K.conv_wgrad(x, D16, Cin, Nout, T, T).view(Nout, Cin)
        wts, wps, wdt = ctx.shapes
        return (dx, dW[:Nt].reshape(wts).to(wdt), db[:Nt].to(wdt), dW[Nt:].reshape(wps).to(wdt),
                db[Nt:].to(wdt))


@K.on_tensor_device
class RtOfflineLayerFunction(torch.autograd.Function):
    """OfflineLayer.forward (models/rtstgcn/rtstgcn.py:343-389) with the Toeplitz matmul it intends
    (rtstgcn.py:366-379) evaluated as the causal K//S-tap box sum it is:

        res = 0 | x | norm_r(conv1x1_nobias(x))
        b   = boxsum_{K,S}( sum_p A_p-mix( conv1x1(x) ) )          (A = A_graph * edge_importance)
        y   = relu(relu(norm(b)) + res)      (residual)     |     relu(norm(b))     (no residual)
    """

    @staticmethod
    def forward(ctx, x, A, wc, bc, nw, nb, wr, nrw, nrb, cfg):
        Kt, S, residual, norm, dtype = cfg[:5]
        sync = cfg[5] if len(cfg) > 5 else None
        bn_finalize = sync.finalize if sync is not None else K.bn_finalize
        dev = x.device
        x = K.to_rows(x, dtype)
        N, Cin, L, V = x.shape
        P = A.shape[-3]
        Cout = wc.shape[0] // P
        M = N * L * V
        A32 = A.detach().float().contiguous()
        res_conv = residual and not (Cin == Cout and S == 1)
        XA, z, _ = gcn_forward(x, A32, wc, bc, dtype)
        b = K.box_sum(z, Kt, S)
        relu_mode = 3 if residual else 2
        r = None
        if res_conv:
            wrp, cq, kq = K.pack_weight(wr.detach().float().view(1, Cout, Cin), dtype)
            if norm == BN:
                str_, _ = gcn_stats_buffer(M, Cout, dev)
            r = K.conv_rows(x, wrp, Cin, Cout, cq, kq, L, L, stats=str_ if norm == BN else None)
        if norm == BN:
            part, nbk, _ = K.bn_stats_partial(b, M, Cout)
            mr, sc, sh = bn_finalize(part, nbk, Cout, Cout, nw.detach().float(), nb.detach().float())
            if res_conv:
                mrr, scr, shr = bn_finalize(str_, str_.shape[0], str_.shape[1], Cout, nrw.detach().float(),
                                              nrb.detach().float())
                y = K.bn_apply(b, sc, sh, M, Cout, res_mode=2, r=r, rsc=scr, rsh=shr, relu=relu_mode)
            else:
                y = K.bn_apply(b, sc, sh, M, Cout, res_mode=1 if residual else 0, r=x if residual else None,
                               relu=relu_mode)
            st, stn = mr, (mrr if res_conv else None)
        else:
            st = K.ln_stats(b, N * L, V, Cout)
            stn = None
            if res_conv:
                stn = K.ln_stats(r, N * L, V, Cout)
                y = K.ln_apply(b, st, _flat_ln(nw), _flat_ln(nb), M, V, Cout, res_mode=2, r=r, rst=stn,
                               rg=_flat_ln(nrw), rb=_flat_ln(nrb), relu=relu_mode)
            else:
                y = K.ln_apply(b, st, _flat_ln(nw), _flat_ln(nb), M, V, Cout, res_mode=1 if residual else 0,
                               r=x if residual else None, relu=relu_mode)
        ctx.cfg = cfg
        ctx.dims = (N, Cin, Cout, L, V, P, res_conv)
        ctx.in_dtype = A.dtype
        saved = [x, A32, XA, b, y, st, wc, bc, nw, nb]
        if norm == BN:
            saved += [sc, sh]
        if res_conv:
            saved += [r, stn, wr, nrw, nrb]
        ctx.save_for_backward(*saved)
        return y

    @staticmethod
    def backward(ctx, dy):
        Kt, S, residual, norm, dtype = ctx.cfg[:5]
        sync = ctx.cfg[5] if len(ctx.cfg) > 5 else None
        N, Cin, Cout, L, V, P, res_conv = ctx.dims
        sv = list(ctx.saved_tensors)
        x, A32, XA, b, y, st, wc, bc, nw, nb = sv[:10]
        rest = sv[10:]
        if norm == BN:
            sc, sh = rest[:2]
            rest = rest[2:]
        if res_conv:
            r, stn, wr, nrw, nrb = rest
        dev = x.device
        M = N * L * V
        dy = K.to_rows(dy, dtype)
        # dq = grad w.r.t. (relu(norm(b)) + res)
        if residual:
            dq = K.cl_empty(N, Cout, L, V, dtype, dev)
            K.bn_bwd_apply(dy, M, Cout, dq, mask=1, mref=y)
        else:
            dq = dy
        dx = K.cl_empty(N, Cin, L, V, dtype, dev)
        dx_written = False
        g = {}
        if res_conv:
            dr = K.cl_empty(N, Cout, L, V, dtype, dev)
            if norm == BN:
                sr = K.bn_bwd_reduce(dq, M, Cout, x=r, mean_rstd=stn)
                g["nrw"], g["nrb"] = sr[:, 1].clone(), sr[:, 0].clone()
                if sync is not None:
                    sync.all_reduce_sums(sr, M)
                K.bn_bwd_apply(dq, M, Cout, dr, x=r, mean_rstd=stn, gamma=nrw.detach().float(), sums=sr)
            else:
                dgbr = torch.zeros((2, Cout * V), dtype=torch.float32, device=dev)
                K.ln_bwd(dq, r, stn, _flat_ln(nrw), _flat_ln(nrb), N * L, V, Cout, dr, dgb=dgbr)
                g["nrw"], g["nrb"] = dgbr[0].view(nrw.shape), dgbr[1].view(nrb.shape)
            wrT, cq, kq = K.pack_weight(wr.detach().float().view(Cout, Cin).t().reshape(1, Cin, Cout), dtype)
            K.conv_rows(dr, wrT, Cout, Cin, cq, kq, L, L, trans=True, out=dx)
            dx_written = True
            g["wr"] = K.conv_wgrad_w(x, dr, Cin, Cout, L, L).view(Cout, Cin, 1, 1)
        elif residual:
            K.bn_bwd_apply(dq, M, Cin, dx)  # dx = dq
            dx_written = True
        # through relu(norm(b))
        db = K.cl_empty(N, Cout, L, V, dtype, dev)
        if norm == BN:
            s1 = K.bn_bwd_reduce(dq, M, Cout, mask=2, mref=b, msc=sc, msh=sh, x=b, mean_rstd=st)
            g["nw"], g["nb"] = s1[:, 1].clone(), s1[:, 0].clone()
            if sync is not None:
                sync.all_reduce_sums(s1, M)
            K.bn_bwd_apply(dq, M, Cout, db, mask=2, mref=b, msc=sc, msh=sh, x=b, mean_rstd=st,
                           gamma=nw.detach().float(), sums=s1)
        else:
            dgb = torch.zeros((2, Cout * V), dtype=torch.float32, device=dev)
            K.ln_bwd(dq, b, st, _flat_ln(nw), _flat_ln(nb), N * L, V, Cout, db, mask=2, dgb=dgb)
            g["nw"], g["nb"] = dgb[0].view(nw.shape), dgb[1].view(nb.shape)
        dz = K.box_sum(db, Kt, S, trans=True)
        dA, dwc, dbc = gcn_backward(x, A32, XA, wc, bc, dz, dx, dx_written, dtype)

        def gr(name, like):
            v = g.get(name)
            return None if v is None or like is None or not like.requires_grad else v.to(like.dtype).view(like.shape)

        return (dx, dA.to(ctx.in_dtype), dwc.to(wc.dtype), dbc.to(bc.dtype), gr("nw", nw), gr("nb", nb),
                gr("wr", wr if res_conv else None), gr("nrw", nrw if res_conv else None),
                gr("nrb", nrb if res_conv else None), None)

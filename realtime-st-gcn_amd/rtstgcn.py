"""RT-ST-GCN (models/rtstgcn/rtstgcn.py) on the HIP kernels.

* ``OfflineLayer`` — training form (rtstgcn.py:220-389): the reference multiplies by an L x L Toeplitz
  matrix and, in this snapshot, crashes on the never-assigned ``self.toeplitz`` (rtstgcn.py:379);
  we evaluate the causal K//S-tap box sum that matrix encodes (rtstgcn.py:368-374), O(K) per output.
* ``OnlineLayer`` + ``AggregateStgcn`` — per-frame inference form (rtstgcn.py:392-627) with the FIFO /
  accumulator state in device buffers (the reference keeps them in CPU tensors, rtstgcn.py:576-579)
  and the step as one HIP kernel (rt.hip).  State is non-persistent (not in the state_dict, exactly
  like the reference's plain attributes).
* ``Model`` — rtstgcn.py:8-217 incl. ``_swap_layers_for_inference`` (rtstgcn.py:160-187).

Stride > 1: offline (K//S taps, dilation S) and online (FIFO of S*(K-1)+1 frames, S accumulators)
diverge in the reference itself (SURVEY §7 hard parts); each form here reproduces its own reference
form (tests/test_gpu_rt.py), and they agree at stride 1.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import layer_fn as LF
from . import native as K
from .routing import ROUTING
from .syncbn import active_sync
from .graph import Graph
from .modules import BatchNorm1d, LayerNorm, make_norm, resolve_dtype
from .stgcn import IN_PAD


class OfflineLayer(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, num_joints, stride, num_partitions, dropout,
                 residual, importance, graph, normalization="LayerNorm"):
        super().__init__()
        assert kernel_size % 2 == 1
        self.num_partitions = num_partitions
        self.num_joints = num_joints
        self.stride = stride
        self.kernel_size = kernel_size
        self.out_channels = out_channels
        self.is_residual = residual
        self.normalization = normalization
        self.dropout = dropout
        self.edge_importance = (nn.Parameter(torch.ones(num_partitions, num_joints, num_joints), requires_grad=True)
                                if importance else 1)
        self.conv = nn.Conv2d(in_channels, out_channels * num_partitions, kernel_size=1)
        self.bn_relu = nn.Sequential(make_norm(normalization, out_channels, num_joints), nn.ReLU())
        self.is_residual_conv = residual and not ((in_channels == out_channels) and (stride == 1))
        if self.is_residual_conv:
            self.residual = nn.Sequential(nn.Conv2d(in_channels, out_channels, kernel_size=1, bias=False),
                                          make_norm(normalization, out_channels, num_joints))
        self.do = nn.Sequential(nn.ReLU(), nn.Dropout(dropout)) if residual else nn.Dropout(dropout)
        self.compute_dtype = torch.float32

    def forward(self, x, A):
        if self.dropout and self.training:
            raise NotImplementedError("stgcn_amd: dropout > 0 in training is not implemented (reference configs use 0)")
        A_eff = A * self.edge_importance
        n = self.bn_relu[0]
        if self.is_residual_conv:
            wr, nrw, nrb = self.residual[0].weight, self.residual[1].weight, self.residual[1].bias
        else:
            wr = nrw = nrb = None
        cfg = (self.kernel_size, self.stride, self.is_residual, self.normalization, self.compute_dtype,
               active_sync(self))
        return LF.RtOfflineLayerFunction.apply(x, A_eff, self.conv.weight, self.conv.bias, n.weight, n.bias, wr,
                                               nrw, nrb, cfg)


class AggregateStgcn(nn.Module):
    """Spatial mix + FIFO temporal aggregation of one frame (rtstgcn.py:556-627).

    forward(x (1, P*C, 1, V) conv output) -> (1, C, 1, V).  ``A`` is this layer's adjacency copy
    (OnlineLayer.eval_ folds the edge importance into it, rtstgcn.py:522-525)."""

    def __init__(self, graph, fifo_size, kernel_size, out_channels, stride):
        super().__init__()
        self.out_channels = out_channels
        self.num_joints = graph.shape[1]
        self.stride = stride
        self.fifo_size = fifo_size
        self.kernel_size = kernel_size
        V = graph.size(1)
        self.register_buffer("A", graph.clone().detach().float(), persistent=False)
        self.register_buffer("fifo", torch.zeros(fifo_size, V, out_channels), persistent=False)
        self.register_buffer("accumulator", torch.zeros(stride, V, out_channels), persistent=False)
        self.register_buffer("idx", torch.zeros(2, dtype=torch.int32), persistent=False)  # (fifo_idx, acc_idx)

    def reset(self):
        self.fifo.zero_()
        self.accumulator.zero_()
        self.idx.zero_()

    def step(self, z):
        """z: (1, C, 1, V) channels-last fp32 frame (already A-mixed and summed over partitions)."""
        out = K.cl_empty(1, self.out_channels, 1, self.num_joints, torch.float32, z.device)
        K.rt_online_step(z, self.fifo, self.accumulator, self.idx, self.out_channels, self.num_joints,
                         self.fifo_size, self.stride, out)
        return out


class OnlineLayer(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, num_joints, stride, num_partitions, dropout,
                 residual, importance, graph, normalization="LayerNorm"):
        super().__init__()
        assert kernel_size % 2 == 1
        fifo_size = stride * (kernel_size - 1) + 1
        self.is_residual = residual
        self.is_residual_conv = residual and not ((in_channels == out_channels) and (stride == 1))
        self.normalization = normalization
        self.edge_importance = (nn.Parameter(torch.ones(num_partitions, num_joints, num_joints), requires_grad=False)
                                if importance else 1)
        self.conv = nn.Conv2d(in_channels, out_channels * num_partitions, kernel_size=1)
        self.aggregate = AggregateStgcn(graph, fifo_size, kernel_size, out_channels, stride)
        self.bn_relu = nn.Sequential(make_norm(normalization, out_channels, num_joints), nn.ReLU())
        if self.is_residual_conv:
            self.residual = nn.Sequential(nn.Conv2d(in_channels, out_channels, kernel_size=1, bias=False),
                                          make_norm(normalization, out_channels, num_joints))
        else:
            self.residual = nn.Identity()
        self.do = nn.Sequential(nn.ReLU(), nn.Dropout(dropout)) if residual else nn.Dropout(dropout)

    def eval_(self):
        self.aggregate.A *= self.edge_importance
        self._packed = None
        return

    def train(self, mode: bool = True):
        """Also drops the per-frame weight packs (see _weights: writes through ``param.data`` are not seen
        by the version counters, so train()/eval()/eval_()/load_state_dict re-pack)."""
        self._packed = None
        return super().train(mode)

    def _load_from_state_dict(self, *args, **kwargs):
        self._packed = None
        return super()._load_from_state_dict(*args, **kwargs)

    def _weights(self, Cin):
        """Per-frame constants (packed GCN weight, A-pushed conv bias, packed residual weight), built once and
        reused while the parameters are unchanged (keyed by their in-place version counters): the per-frame
        step then launches only data-dependent kernels."""
        A = self.aggregate.A
        rw = self.residual[0].weight if self.is_residual_conv else None
        key = (A.data_ptr(), A._version, self.conv.weight.data_ptr(), self.conv.weight._version,
               self.conv.bias.data_ptr(), self.conv.bias._version,
               None if rw is None else (rw.data_ptr(), rw._version))
        pk = getattr(self, "_packed", None)
        if pk is not None and pk[0] == key:
            return pk[1]
        P = A.shape[0]
        Cout = self.aggregate.out_channels
        A32 = A.detach().float().contiguous()
        wg3 = self.conv.weight.detach().float().view(P, Cout, Cin).permute(1, 0, 2).reshape(1, Cout, P * Cin)
        wgp, cp, kp = K.pack_weight(wg3, torch.float32)
        bias2d = K.gcn_bias(A32, self.conv.bias.detach().float().contiguous(), 1, Cout)
        res = K.pack_weight(rw.detach().float().view(1, Cout, Cin), torch.float32) if rw is not None else None
        packed = (A32, wgp, cp, kp, bias2d, res)
        self._packed = (key, packed)
        return packed

    @torch.no_grad()
    def forward(self, x, A):
        x = K.to_rows(x, torch.float32)
        if x.shape[0] != 1 or x.shape[2] != 1:
            raise RuntimeError("OnlineLayer processes one frame of batch 1 (rtstgcn.py:607)")
        V = x.shape[3]
        Cout = self.aggregate.out_channels
        P = self.aggregate.A.shape[0]
        Cin = x.shape[1]
        A32, wgp, cp, kp, bias2d, resp = self._weights(Cin)
        ag = self.aggregate
        if self.normalization == "LayerNorm" and x.shape[1] % 4 == 0 and V <= 32 and P <= 3 and Cin <= 256:
            # one frame in 2 launches (rt_fused.hip): conv1x1 + A-mix + FIFO (+ residual conv), then the norms
            wr = self.residual[0].weight if self.is_residual_conv else None
            a, r = K.rt_frame_gcn(x, A32, self.conv.weight.detach(), bias2d, ag.fifo, ag.accumulator, ag.idx,
                                  None if wr is None else wr.detach())
            n = self.bn_relu[0]
            res_mode = 2 if self.is_residual_conv else (1 if self.is_residual else 0)
            rn = self.residual[1] if self.is_residual_conv else None
            return K.rt_frame_norm(a, LF._flat_ln(n.weight), LF._flat_ln(n.bias), res_mode,
                                   r if self.is_residual_conv else (x if self.is_residual else None),
                                   None if rn is None else LF._flat_ln(rn.weight),
                                   None if rn is None else LF._flat_ln(rn.bias), ag.idx, ag.fifo_size, ag.stride)
        XA = K.amix_fwd(x, A32)
        z = K.conv_rows(XA, wgp, P * Cin, Cout, cp, kp, 1, 1, bias=bias2d, bias_mode=2)
        a = self.aggregate.step(z)
        n = self.bn_relu[0]
        relu_mode = 3 if self.is_residual else 2
        if self.is_residual_conv:
            wrp, cq, kq = resp
            r = K.conv_rows(x, wrp, Cin, Cout, cq, kq, 1, 1)
        res_mode = 2 if self.is_residual_conv else (1 if self.is_residual else 0)
        res = r if self.is_residual_conv else (x if self.is_residual else None)
        if self.normalization == "LayerNorm":
            st = K.ln_stats(a, 1, V, Cout)
            rst = rg = rb = None
            if self.is_residual_conv:
                rst = K.ln_stats(r, 1, V, Cout)
                rg, rb = LF._flat_ln(self.residual[1].weight), LF._flat_ln(self.residual[1].bias)
            return K.ln_apply(a, st, LF._flat_ln(n.weight), LF._flat_ln(n.bias), V, V, Cout, res_mode=res_mode,
                              r=res, rst=rst, rg=rg, rb=rb, relu=relu_mode)
        # batch-statistics BatchNorm over the V joints of the frame
        part, nb, _ = K.bn_stats_partial(a, V, Cout)
        _, sc, sh = K.bn_finalize(part, nb, Cout, Cout, n.weight.float(), n.bias.float())
        rsc = rsh = None
        if self.is_residual_conv:
            rpart, rnb, _ = K.bn_stats_partial(r, V, Cout)
            _, rsc, rsh = K.bn_finalize(rpart, rnb, Cout, Cout, self.residual[1].weight.float(),
                                        self.residual[1].bias.float())
        return K.bn_apply(a, sc, sh, V, Cout, res_mode=res_mode, r=res, rsc=rsc, rsh=rsh, relu=relu_mode)


class Model(nn.Module):
    """rt-st-gcn (rtstgcn.py:8-217): forward(x (N, C, L, V)) -> (N, num_classes, L)."""

    def __init__(self, rank=None, **kwargs):
        super().__init__()
        self.conf = kwargs["rt-st-gcn"]
        self.graph = Graph(strategy=kwargs["strategy"], **kwargs["graph"])
        # contiguous: graph.A is a transposed view (graph.py:179) and torch.tensor keeps its strides, so every
        # A * edge_importance product (and each layer's dense copy of it) would be permuted
        A = torch.tensor(self.graph.A, dtype=torch.float32, requires_grad=False).contiguous()
        self.register_buffer("A", A)
        self.normalization = kwargs["normalization"]
        self.norm_in = (LayerNorm([kwargs["in_feat"], 1, A.size(1)]) if kwargs["normalization"] == "LayerNorm"
                        else BatchNorm1d(kwargs["in_feat"] * A.size(1), track_running_stats=False))
        self.fcn_in = nn.Conv2d(in_channels=self.conf["in_feat"], out_channels=self.conf["in_ch"][0], kernel_size=1)
        self.st_gcn = nn.ModuleList([self._layer(OfflineLayer, i, kwargs["graph"]["num_node"])
                                     for i in range(self.conf["layers"])])
        self.avg_pool = nn.AvgPool2d(kernel_size=(1, kwargs["graph"]["num_node"]))
        self.fcn_out = nn.Conv2d(in_channels=self.conf["out_ch"][-1], out_channels=kwargs["num_classes"],
                                 kernel_size=1)
        self.compute_dtype = torch.float32
        self.online = False

    def _layer(self, cls, i, V):
        return cls(num_joints=V, in_channels=self.conf["in_ch"][i], out_channels=self.conf["out_ch"][i],
                   kernel_size=self.conf["kernel"], stride=self.conf["stride"][i], num_partitions=self.A.shape[0],
                   residual=not not self.conf["residual"][i], dropout=self.conf["dropout"][i],
                   importance=self.conf["importance"], graph=self.A, normalization=self.normalization)

    def set_compute_dtype(self, dtype):
        dt = resolve_dtype(dtype)
        self.compute_dtype = dt
        for layer in self.st_gcn:
            if hasattr(layer, "compute_dtype"):
                layer.compute_dtype = dt
        return self

    def forward(self, x):
        if (self.online and self.normalization == "LayerNorm" and x.dim() == 4 and x.shape[0] == 1
                and x.shape[2] == 1 and x.shape[1] == 3 and not torch.is_grad_enabled()):
            if ROUTING.rt_one_launch and self._frame_desc_ok():
                # the whole frame as ONE persistent launch (rt_fused.hip rt_frame_kernel)
                return self._rt_frame(x)
            # per-frame inference: fused input head, two launches per layer, fused output head (rt_fused.hip)
            y = K.rt_frame_in(x, LF._flat_ln(self.norm_in.weight), LF._flat_ln(self.norm_in.bias),
                              self.fcn_in.weight.detach().reshape(self.fcn_in.out_channels, -1),
                              self.fcn_in.bias.detach())
            for gcn in self.st_gcn:
                y = gcn(y, self.A)
            return K.rt_frame_out(y, self.fcn_out.weight.detach().reshape(self.fcn_out.out_channels, -1),
                                  self.fcn_out.bias.detach())
        x = self.norm_in(x)
        C = x.shape[1]
        if C % IN_PAD:
            x = F.pad(x.permute(0, 2, 3, 1), (0, IN_PAD - C % IN_PAD)).permute(0, 3, 1, 2)
            w = F.pad(self.fcn_in.weight, (0, 0, 0, 0, 0, IN_PAD - C % IN_PAD))
        else:
            w = self.fcn_in.weight
        dt = torch.float32 if self.online else self.compute_dtype
        x = LF.Conv1x1Function.apply(x, w, self.fcn_in.bias, dt)
        for gcn in self.st_gcn:
            x = gcn(x, self.A)
        x = LF.PoolFunction.apply(x, dt, True)
        x = LF.Conv1x1Function.apply(x, self.fcn_out.weight, self.fcn_out.bias, dt)
        return x.squeeze(-1).float()

    def _frame_desc_ok(self):
        """Shapes the one-launch frame kernel takes (stgcn_rt_frame): LayerNorm online layers, C % 4 == 0, C <= 256,
        V <= 32, V * C <= 7680, P <= 3, at most 12 layers."""
        V = self.A.shape[-1]
        if not (2 <= V <= 32 and len(self.st_gcn) <= K.L.RT_MAX_LAYERS and self.fcn_in.out_channels % 4 == 0):
            return False
        for l in self.st_gcn:
            if not isinstance(l, OnlineLayer) or l.normalization != "LayerNorm" or l.aggregate.A.shape[0] > 3:
                return False
            C = l.aggregate.out_channels
            if l.conv.in_channels % 4 or C % 4 or C > 256 or V * C > 7680:
                return False
        return True

    def _frame_key(self):
        """Key of the frame descriptor: data pointers and in-place versions of every parameter it reads (copies of
        them live in the descriptor), data pointers only of the FIFO state (the kernel updates it in place, and
        reset_state's zeroing must not rebuild the descriptor)."""
        ts = [self.norm_in.weight, self.norm_in.bias, self.fcn_in.weight, self.fcn_in.bias, self.fcn_out.weight,
              self.fcn_out.bias]
        st = []
        for l in self.st_gcn:
            ts += [l.aggregate.A, l.conv.weight, l.conv.bias, l.bn_relu[0].weight, l.bn_relu[0].bias]
            st += [l.aggregate.fifo, l.aggregate.accumulator, l.aggregate.idx]
            if l.is_residual_conv:
                ts += [l.residual[0].weight, l.residual[1].weight, l.residual[1].bias]
        return tuple((t.data_ptr(), t._version) for t in ts) + tuple(t.data_ptr() for t in st)

    def _rt_frame(self, x):
        key = self._frame_key()
        pk = getattr(self, "_frame_pack", None)
        if pk is None or pk[0] != key:
            pk = (key, self._build_frame_desc())
            self._frame_pack = pk
        desc, _keep = pk[1]
        out = torch.empty((1, self.fcn_out.out_channels, 1), dtype=torch.float32, device=x.device)
        return K.rt_frame(desc, x, out)

    def _build_frame_desc(self):
        """stgcn_rt_frame_desc of this model (K.L.RtFrameDesc) + the tensors it points to (kept alive with it)."""
        V = self.A.shape[-1]
        dev = self.A.device
        keep = []

        def p(t):
            keep.append(t)
            return t.data_ptr()

        d = K.L.RtFrameDesc()
        d.V, d.L, d.C0, d.K, d.blocks = V, len(self.st_gcn), self.fcn_in.out_channels, self.fcn_out.out_channels, 0
        d.ln_w, d.ln_b = p(LF._flat_ln(self.norm_in.weight)), p(LF._flat_ln(self.norm_in.bias))
        d.w_in = p(self.fcn_in.weight.detach().float().reshape(self.fcn_in.out_channels, -1).contiguous())
        d.b_in = p(self.fcn_in.bias.detach().float().contiguous())
        d.w_out = p(self.fcn_out.weight.detach().float().reshape(self.fcn_out.out_channels, -1).contiguous())
        d.b_out = p(self.fcn_out.bias.detach().float().contiguous())
        d.sync = p(torch.zeros(4, dtype=torch.int32, device=dev))
        self._frame_status = torch.zeros(1, dtype=torch.int32, device=dev)
        d.status = p(self._frame_status)
        for i, l in enumerate(self.st_gcn):
            ag = l.aggregate
            Cin, Cout = l.conv.in_channels, ag.out_channels
            A32, _, _, _, bias2d, _ = l._weights(Cin)
            y = d.layers[i]
            y.Cin, y.Cout, y.P, y.fifo_size, y.S = Cin, Cout, ag.A.shape[0], ag.fifo_size, ag.stride
            y.res_mode = 2 if l.is_residual_conv else (1 if l.is_residual else 0)
            y.A, y.w, y.bias2d = p(A32), p(l.conv.weight.detach().float().contiguous()), p(bias2d)
            n = l.bn_relu[0]

            def rows(t):  # LayerNorm([C,1,V]) affine (C,1,V) -> the rows' [V][C] layout
                return t.detach().float().reshape(Cout, V).t().contiguous()

            y.ln_w, y.ln_b = p(rows(n.weight)), p(rows(n.bias))
            y.fifo, y.acc, y.idx = p(ag.fifo), p(ag.accumulator), p(ag.idx)
            y.a_buf = p(torch.empty(V * Cout, dtype=torch.float32, device=dev))
            if l.is_residual_conv:
                y.wr = p(l.residual[0].weight.detach().float().reshape(Cout, Cin).contiguous())
                y.lnr_w, y.lnr_b = p(rows(l.residual[1].weight)), p(rows(l.residual[1].bias))
                y.r_buf = p(torch.empty(V * Cout, dtype=torch.float32, device=dev))
        return d, keep

    def _swap_layers_for_inference(self):
        """Replace OfflineLayers by OnlineLayers carrying the same parameters (rtstgcn.py:160-187)."""
        V = self.A.shape[-1]
        new = nn.ModuleList([self._layer(OnlineLayer, i, V) for i in range(self.conf["layers"])])
        new.load_state_dict(self.st_gcn.state_dict(), strict=False)
        self.st_gcn = new.to(self.A.device)
        self.online = True
        return

    def reset_state(self):
        for layer in self.st_gcn:
            if isinstance(layer, OnlineLayer):
                layer.aggregate.reset()

    def prepare_benchmark(self, arch_conf):
        """Intended semantics of rtstgcn.py:190-197 (which calls a missing method): swap to online layers
        and fold the edge importance (OnlineLayer.eval_)."""
        self._swap_layers_for_inference()
        for module in self.st_gcn:
            module.eval_()
        return arch_conf

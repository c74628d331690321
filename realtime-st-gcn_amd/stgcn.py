"""ST-GCN classifier (models/stgcn/stgcn.py:8-101) on the HIP kernels.

``Model(**arch)`` takes the reference's ``arch`` config dict (+ injected ``graph`` and
``num_classes``, processor.py:164-166); ``rank`` is accepted and ignored like in the reference.
state_dict keys are identical (``A``, ``norm_in.*``, ``fcn_in.*``, ``gcn_networks.i.*``,
``edge_importance.i``, ``fcn_out.*``).  forward(x (N, C, T, V)) -> (N, num_classes, 1); x may also be a
``segment.WindowBatch`` (WindowSegment's sliding windows over a padded capture), whose norm_in + fcn_in
run from the capture without forming the windows (layer_fn.WindowStageFunction).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import layer_fn as LF
from . import native as K
from .graph import Graph
from .modules import BatchNorm1d, LayerNorm, StgcnLayer, resolve_dtype
from .routing import ROUTING
from .segment import WindowBatch

IN_PAD = 8  # fcn_in input channels are zero-padded to one 16-byte unit (kernel vector width)


class Model(nn.Module):
    def __init__(self, rank=None, **kwargs):
        super().__init__()
        conf = kwargs["st-gcn"]
        self.graph = Graph(strategy=kwargs["strategy"], **kwargs["graph"])
        # contiguous: graph.A is a transposed view (graph.py:179) and torch.tensor keeps its strides, so every
        # A * edge_importance product (and each layer's dense copy of it) would be permuted
        A = torch.tensor(self.graph.A, dtype=torch.float32, requires_grad=False).contiguous()
        self.register_buffer("A", A)
        kernel_size = (conf["kernel"], kwargs["graph"]["num_node"])
        self.normalization = kwargs["normalization"]
        self.norm_in = (LayerNorm([kwargs["in_feat"], 1, A.size(1)]) if kwargs["normalization"] == "LayerNorm"
                        else BatchNorm1d(kwargs["in_feat"] * A.size(1), track_running_stats=False))
        self.fcn_in = nn.Conv2d(in_channels=conf["in_feat"], out_channels=conf["in_ch"][0], kernel_size=1)
        self.gcn_networks = nn.ModuleList([
            StgcnLayer(in_channels=conf["in_ch"][i], out_channels=conf["out_ch"][i], kernel_size=kernel_size,
                       partitions=A.size(0), num_joints=A.size(1), stride=conf["stride"][i],
                       residual=not not conf["residual"][i], dropout=conf["dropout"][i],
                       normalization=kwargs["normalization"])
            for i in range(conf["layers"])])
        if conf["importance"]:
            self.edge_importance = nn.ParameterList([nn.Parameter(torch.ones(self.A.size()))
                                                     for _ in self.gcn_networks])
        else:
            self.edge_importance = [1] * len(self.gcn_networks)
        self.fcn_out = nn.Conv2d(conf["out_ch"][-1], out_channels=kwargs["num_classes"], kernel_size=1)
        self.compute_dtype = torch.float32
        self._plan = None  # native.PrepPlan of the training forward (not state: rebuilt when storages move)

    def set_compute_dtype(self, dtype):
        """fp32 (parity) or bf16 (perf) arithmetic for every layer; the input norm stays fp32."""
        dt = resolve_dtype(dtype)
        self.compute_dtype = dt
        for layer in self.gcn_networks:
            for m in layer.modules():
                if hasattr(m, "compute_dtype"):
                    m.compute_dtype = dt
        return self

    def _prepared(self):
        """Every packed operand of the training step (the layers' graph-conv effective weights with the bias
        through A, temporal / residual / head conv packs, forward and data-gradient forms) in ONE launch
        (native.PrepPlan, prep.hip) instead of ~50 per-layer launches; returns the plan (its ``layers`` /
        ``head`` packs) or None.  Only for the autograd path on the device: inference keeps the per-call
        packing (the fused inference route packs differently).  The packs are refilled every forward from the
        current parameters; the plan (job table of raw pointers) is rebuilt when a storage moves.
        nn.DataParallel replicas (the reference's multi-GPU form, processor.py:33) are rebuilt every forward
        from freshly broadcast storages, so a plan would be rebuilt per step and never reach the parent: they
        pack per call instead."""
        if not (ROUTING.prep_plan and torch.is_grad_enabled() and self.A.is_cuda) or getattr(self, "_is_replica",
                                                                                              False):
            return None
        dt = self.compute_dtype
        imp = isinstance(self.edge_importance, nn.ParameterList) and len(self.edge_importance)
        key = (dt, self.A.data_ptr(), tuple(p.data_ptr() for p in self.parameters()))
        plan = self._plan
        if plan is None or plan.key != key:
            with K.device_of(self.A):
                plan = K.PrepPlan(self.A.device, key)
                plan.layers = []
                for i, gcn in enumerate(self.gcn_networks):
                    gcn.bind_graph(self.A)
                    plan.layers.append(LF.plan_layer_packs(plan, gcn, self.A, self.edge_importance[i] if imp else None,
                                                           dt))
                plan.head = (LF.plan_conv1x1_packs(plan, self.fcn_in.weight, dt),
                             LF.plan_conv1x1_packs(plan, self.fcn_out.weight, dt))
                plan.finalize()
            self._plan = plan
        with K.device_of(self.A):
            plan.run()
        return plan

    def stage_windows(self, xb: WindowBatch):
        """norm_in + fcn_in (stgcn.py:82-85) of sliding windows, from the padded capture."""
        return LF.stage_window_batch(xb, self.norm_in, self.fcn_in, self.compute_dtype)

    def forward(self, x):
        plan = self._prepared()
        if isinstance(x, WindowBatch):
            x = self.stage_windows(x)
        else:
            x = self.norm_in(x)                                          # stgcn.py:82 (fp32)
            C = x.shape[1]
            if C % IN_PAD:  # rows of one 16-byte unit; the weight's missing input columns act as zeros
                x = F.pad(x.permute(0, 2, 3, 1), (0, IN_PAD - C % IN_PAD)).permute(0, 3, 1, 2)
            x = LF.Conv1x1Function.apply(x, self.fcn_in.weight, self.fcn_in.bias, self.compute_dtype,
                                         plan.head[0] if plan is not None else None)   # stgcn.py:85
        if isinstance(self.edge_importance, nn.ParameterList) and len(self.edge_importance):
            # A * M_i of every layer as one stacked product (one launch each way instead of one per layer)
            A_eff = (self.A * torch.stack(list(self.edge_importance))).unbind(0)
        else:
            A_eff = [self.A * m for m in self.edge_importance]
        for i, (gcn, A_i) in enumerate(zip(self.gcn_networks, A_eff)):                 # stgcn.py:88-89
            gcn.bind_graph(self.A)  # support of the static graph (cached; no sync after the first call)
            x = gcn(x, A_i, packs=plan.layers[i] if plan is not None else None)
        x = LF.PoolFunction.apply(x, self.compute_dtype)                            # stgcn.py:92
        x = LF.Conv1x1Function.apply(x, self.fcn_out.weight, self.fcn_out.bias, self.compute_dtype,
                                     plan.head[1] if plan is not None else None)  # :95
        return x.squeeze(-1).float()                                                # :97

    def prepare_benchmark(self, arch_conf):
        return arch_conf

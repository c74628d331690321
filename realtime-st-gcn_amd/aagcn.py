"""AAGCN (models/aagcn/aagcn.py) on the HIP kernels: two streams (joints, bones), each an ST-GCN whose
layers use the adjacency A + B + C with C = softmax(theta^T phi) a per-sample attention matrix.

The per-sample (N, P, V, V) adjacency runs through the same HIP graph-conv kernels as the shared one
(per_sample mode of amix/gcn_bias, tgcn.py:69-78 broadcasting); the attention scores run on MFMA
(attn.hip).  state_dict keys match the reference (``streams.{0,1}.{norm_in,fcn_in,gcn_networks,fcn_out}``,
``...gcn_networks.i.{B, theta, phi, st_gcn.*}``).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import layer_fn as LF
from .graph import Graph
from .modules import BatchNorm1d, LayerNorm, StgcnLayer, resolve_dtype
from .segment import WindowBatch
from .stgcn import IN_PAD


class AgcnLayer(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, partitions, stride, residual, dropout, num_joints,
                 normalization="LayerNorm"):
        super().__init__()
        coeff_embedding = 4
        self.embedding_channels = out_channels // coeff_embedding
        self.partitions = partitions
        self.num_joints = num_joints
        self.B = nn.Parameter(torch.zeros(partitions, num_joints, num_joints), requires_grad=True)
        self.theta = nn.Conv2d(in_channels, self.embedding_channels * partitions, 1)
        self.phi = nn.Conv2d(in_channels, self.embedding_channels * partitions, 1)
        self.st_gcn = StgcnLayer(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                                 partitions=partitions, num_joints=num_joints, stride=stride, dropout=dropout,
                                 residual=residual, normalization=normalization)
        self.compute_dtype = torch.float32

    def forward(self, x, A):
        # The attention logits theta^T phi contract over C'*T (4800 terms at config 5) and feed a softmax:
        # with bf16-stored theta/phi their rounding moves the logits by O(0.1) and the softmax weights by
        # O(10 %), so this branch runs in fp32 on every compute dtype (it is ~3 % of the layer's work).
        att = torch.float32
        Cin = self.theta.weight.shape[1]
        if LF.attn_proj_ok(x, Cin, self.theta.weight.shape[0], self.phi.weight.shape[0], self.compute_dtype):
            # bf16 model: fp32 theta/phi straight from the bf16 activation (attn_proj, W split hi + lo)
            theta, phi = LF.AttnProjFunction.apply(x, self.theta.weight, self.theta.bias, self.phi.weight,
                                                   self.phi.bias)
        else:
            theta = LF.Conv1x1Function.apply(x, self.theta.weight, self.theta.bias, att)
            phi = LF.Conv1x1Function.apply(x, self.phi.weight, self.phi.bias, att)
        C = LF.AttentionFunction.apply(theta, phi, self.partitions, att)         # (N, P, V, V)
        return self.st_gcn(x, A + self.B + C)                                    # aagcn.py:148


class Model(nn.Module):
    """aa-gcn (aagcn.py:8-95): forward(x (N, C, T, V)) -> (N, num_classes)."""

    def __init__(self, rank=None, **kwargs):
        super().__init__()
        conf = kwargs["aa-gcn"]
        self.graph = Graph(strategy=kwargs["strategy"], **kwargs["graph"])
        # contiguous: graph.A is a transposed view (graph.py:179) and torch.tensor keeps its strides, so every
        # A * edge_importance product (and each layer's dense copy of it) would be permuted
        A = torch.tensor(self.graph.A, dtype=torch.float32, requires_grad=False).contiguous()
        self.register_buffer("A", A)
        kernel_size = (conf["kernel"], kwargs["graph"]["num_node"])
        self.num_classes = kwargs["num_classes"]
        self.streams = nn.ModuleList([nn.ModuleDict({
            "norm_in": (LayerNorm([kwargs["in_feat"], 1, A.size(1)]) if kwargs["normalization"] == "LayerNorm"
                        else BatchNorm1d(kwargs["in_feat"] * A.size(1), track_running_stats=False)),
            "fcn_in": nn.Conv2d(in_channels=conf["in_feat"], out_channels=conf["in_ch"][0], kernel_size=1),
            "gcn_networks": nn.ModuleList([
                AgcnLayer(in_channels=conf["in_ch"][i], out_channels=conf["out_ch"][i], kernel_size=kernel_size,
                          partitions=A.size(0), stride=conf["stride"][i], residual=not not conf["residual"][i],
                          dropout=conf["dropout"][i], num_joints=kwargs["graph"]["num_node"],
                          normalization=kwargs["normalization"])
                for i in range(conf["layers"])]),
            "fcn_out": nn.Conv2d(in_channels=conf["out_ch"][-1], out_channels=kwargs["num_classes"], kernel_size=1),
        }) for _ in ["joints", "bones"]])
        ot = kwargs["output_type"]
        self.output_type = ot
        # bone construction: for each joint i, its "far" neighbours j get x[j] - x[i] (aagcn.py:63-68)
        far = self.graph.get_adjacency_raw()[2].astype(bool)
        src = np.zeros(A.size(1), dtype=np.int64)
        has = np.zeros(A.size(1), dtype=bool)
        for i in range(A.size(1)):  # later i overwrite earlier ones, as in the reference loop
            for j in np.nonzero(far[i])[0]:
                src[j] = i
                has[j] = True
        self.register_buffer("bone_src", torch.tensor(src), persistent=False)
        self.register_buffer("bone_mask", torch.tensor(has, dtype=torch.float32), persistent=False)
        self.compute_dtype = torch.float32

    def set_compute_dtype(self, dtype):
        dt = resolve_dtype(dtype)
        self.compute_dtype = dt
        for s in self.streams:
            for layer in s["gcn_networks"]:
                for m in layer.modules():
                    if hasattr(m, "compute_dtype"):
                        m.compute_dtype = dt
        return self

    def probability(self, x):
        if self.output_type == "logsoftmax":
            return F.log_softmax(x, dim=1)
        if self.output_type == "softmax":
            return F.softmax(x, dim=1)
        return x

    def _stream(self, s, x):
        if isinstance(x, WindowBatch):  # sliding windows staged from the capture (window.hip)
            x = LF.stage_window_batch(x, s["norm_in"], s["fcn_in"], self.compute_dtype)
        else:
            x = s["norm_in"](x)
            C = x.shape[1]
            w = s["fcn_in"].weight
            if C % IN_PAD:
                x = F.pad(x.permute(0, 2, 3, 1), (0, IN_PAD - C % IN_PAD)).permute(0, 3, 1, 2)
                w = F.pad(w, (0, 0, 0, 0, 0, IN_PAD - C % IN_PAD))
            x = LF.Conv1x1Function.apply(x, w, s["fcn_in"].bias, self.compute_dtype)
        for gcn in s["gcn_networks"]:
            x = gcn(x, self.A)
        x = LF.PoolFunction.apply(x, self.compute_dtype)
        x = LF.Conv1x1Function.apply(x, s["fcn_out"].weight, s["fcn_out"].bias, self.compute_dtype)
        return x.squeeze(-1).float()

    def forward(self, x_joint):
        # bones: x_bone[..., j] = x[..., j] - x[..., src(j)] for joints that are someone's far neighbour;
        # a per-frame map, so a WindowBatch's bone windows are the windows of the capture's bones
        if isinstance(x_joint, WindowBatch):
            cap = x_joint.capture
            x_bone = WindowBatch((cap - cap[:, :, :, self.bone_src]) * self.bone_mask, x_joint.n0, x_joint.nw,
                                 x_joint.W)
        else:
            x_bone = (x_joint - x_joint[:, :, :, self.bone_src]) * self.bone_mask
        y_joint = self._stream(self.streams[0], x_joint)
        y_bone = self._stream(self.streams[1], x_bone)
        return self.probability(y_bone) + self.probability(y_joint)            # aagcn.py:95

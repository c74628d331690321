"""CPU ORACLE — test infrastructure only, never the product.

A from-scratch, functional CPU restatement (numpy for the host-side graph,
PyTorch-CPU fp32/fp64 for the floating-point layer math) of the reference's
ST-GCN hot path.  Every function cites the reference file:line it restates.

Who may import this file: ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — and only as the checker / the timed
CPU baseline.  The product package (``realtime-st-gcn_amd/``) never imports it
and has no CPU fallback.

Pinning: every function here is checked against the golden fixtures in
``tests/golden/*.npz``, which were produced by running the reference itself
in the build container (``tests/golden/make_golden.py``).  See
``tests/test_oracle_golden.py``.

Tensors use the reference's logical layout (N, C, T, V).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# --------------------------------------------------------------------------------------
# Graph (host side, numpy fp64)  — models/utils/graph.py
# --------------------------------------------------------------------------------------


def hop_distance(num_node, edge):
    """All-pairs hop distance by Floyd-Warshall (graph.py:182-205)."""
    d = np.full((num_node, num_node), np.inf)
    for i, j in edge:
        if i == j:
            d[i, i] = 0
        else:
            d[i, j] = d[j, i] = 1
    for k in range(num_node):
        d = np.minimum(d, d[:, k:k + 1] + d[k:k + 1, :])
    return d


def adjacency(num_node, edge, center, strategy="spatial", max_hop=1, dilation=1):
    """Partitioned 0/1 adjacency (graph.py:108-170).  'uniform' is all zeros (graph.py:134-135)."""
    hop = hop_distance(num_node, edge)
    valid = list(range(0, max_hop + 1, dilation))
    adj = np.zeros((num_node, num_node))
    for h in valid:
        adj[hop == h] = 1
    if strategy == "uniform":
        return np.zeros((1, num_node, num_node))
    if strategy == "distance":
        A = np.zeros((len(valid), num_node, num_node))
        for i, h in enumerate(valid):
            A[i][hop == h] = adj[hop == h]
        return A
    if strategy != "spatial":
        raise ValueError("Strategy Does Not Exist.")
    dc = hop[:, center]
    parts = []
    for h in valid:
        on = hop == h
        root = np.where(on & (dc[None, :] == dc[:, None]), adj, 0.0)
        close = np.where(on & (dc[None, :] < dc[:, None]), adj, 0.0)
        far = np.where(on & (dc[None, :] > dc[:, None]), adj, 0.0)
        if h == 0:
            parts.append(root)
        else:
            parts += [close, far]
    return np.stack(parts)


def normalize(A, alpha=0.001, symmetric=True):
    """Per-partition degree normalisation then transpose (graph.py:173-179, 208-243)."""
    out = np.empty_like(A)
    for i in range(A.shape[0]):
        deg = A[i].sum(1) + alpha
        if symmetric:
            dl = np.power(deg, -0.5)
            dl[np.isinf(dl)] = 0
            out[i] = dl[:, None] * A[i] * dl[None, :]
        else:
            dl = np.power(deg, -1.0)
            dl[np.isinf(dl)] = 0
            out[i] = A[i] * dl[None, :]
    return out.transpose(0, 2, 1)


def graph_A(num_node, edge, center, strategy="spatial", normalization="symmetric", max_hop=1, dilation=1,
            alpha=0.001):
    """``Graph(...).A`` (graph.py:33-89)."""
    return normalize(adjacency(num_node, edge, center, strategy, max_hop, dilation), alpha,
                     normalization == "symmetric")


# --------------------------------------------------------------------------------------
# Norms — models/utils/layernorm.py, models/utils/batchnorm.py, nn.BatchNorm2d(track_running_stats=False)
# --------------------------------------------------------------------------------------


def layernorm_cv(x, weight, bias, eps=1e-5):
    """Custom LayerNorm([C,1,V]) over (C,V) per (n,t), UNBIASED var (layernorm.py:22-28)."""
    mean = x.mean(dim=(1, 3), keepdim=True)
    var = x.var(dim=(1, 3), keepdim=True, unbiased=True)
    return weight * ((x - mean) / torch.sqrt(var + eps)) + bias


def batchnorm_batch(x, weight, bias, eps=1e-5):
    """BatchNorm2d(C, track_running_stats=False): batch stats over (N,T,V), biased var (stgcn.py:152)."""
    mean = x.mean(dim=(0, 2, 3), keepdim=True)
    var = x.var(dim=(0, 2, 3), keepdim=True, unbiased=False)
    return (x - mean) / torch.sqrt(var + eps) * weight.view(1, -1, 1, 1) + bias.view(1, -1, 1, 1)


def input_batchnorm(x, weight, bias, eps=1e-5):
    """BatchNorm1d(C*V) on (N, V*C, T): stats per (v,c) over (N,T) (batchnorm.py:13-23).

    ``weight``/``bias`` are indexed by v*C + c.
    """
    N, C, T, V = x.shape
    xp = x.permute(0, 3, 1, 2).reshape(N, V * C, T)
    mean = xp.mean(dim=(0, 2), keepdim=True)
    var = xp.var(dim=(0, 2), keepdim=True, unbiased=False)
    y = (xp - mean) / torch.sqrt(var + eps) * weight.view(1, -1, 1) + bias.view(1, -1, 1)
    return y.view(N, V, C, T).permute(0, 2, 3, 1)


def norm(kind, x, w, b):
    return layernorm_cv(x, w, b) if kind == "LayerNorm" else batchnorm_batch(x, w, b)


# --------------------------------------------------------------------------------------
# Graph convolution — models/utils/tgcn.py:58-79
# --------------------------------------------------------------------------------------


def tgcn(x, weight, bias, A):
    """1x1 conv (C_in -> P*C_out, WITH bias) then matmul with A over V, summed over P.

    A is (P,V,V) or per-sample (N,P,V,V) (tgcn.py:69-78).
    """
    N, _, T, V = x.shape
    P = A.shape[-3]
    C = weight.shape[0] // P
    z = F.conv2d(x, weight, bias)
    z = z.view(N, P, C * T, V)
    y = torch.matmul(z, A)
    return y.sum(dim=1).view(N, C, T, V)


# --------------------------------------------------------------------------------------
# StgcnLayer — models/stgcn/stgcn.py:104-193
# --------------------------------------------------------------------------------------


def stgcn_layer(x, A, sd, prefix, kt, stride, residual, normalization):
    """StgcnLayer.forward (stgcn.py:181-193).  ``sd`` holds the reference state_dict names."""
    g = lambda k: sd[prefix + k]  # noqa: E731
    cin, cout = x.shape[1], g("tcn.2.weight").shape[0]
    pad = (kt - 1) // 2
    if not residual:
        res = x * 0.0
    elif cin == cout and stride == 1:
        res = x
    else:
        r = F.conv2d(x, g("residual.0.weight"), g("residual.0.bias"), stride=(stride, 1))
        res = norm(normalization, r, g("residual.1.weight"), g("residual.1.bias"))
    h = tgcn(x, g("gcn.conv.weight"), g("gcn.conv.bias"), A)
    h = torch.relu(norm(normalization, h, g("tcn.0.weight"), g("tcn.0.bias")))
    h = F.conv2d(h, g("tcn.2.weight"), g("tcn.2.bias"), stride=(stride, 1), padding=(pad, 0))
    h = norm(normalization, h, g("tcn.3.weight"), g("tcn.3.bias"))
    return torch.relu(h + res)


def stgcn_model(x, sd, arch):
    """st-gcn Model.forward (stgcn.py:80-97) with ``arch`` = config 'arch' + graph + num_classes."""
    conf = arch["st-gcn"]
    kind = arch["normalization"]
    if kind == "LayerNorm":
        x = layernorm_cv(x, sd["norm_in.weight"], sd["norm_in.bias"])
    else:
        x = input_batchnorm(x, sd["norm_in.norm.weight"], sd["norm_in.norm.bias"])
    x = F.conv2d(x, sd["fcn_in.weight"], sd["fcn_in.bias"])
    A = sd["A"]
    for i in range(conf["layers"]):
        Ai = A * sd["edge_importance.%d" % i] if conf["importance"] else A
        x = stgcn_layer(x, Ai, sd, "gcn_networks.%d." % i, conf["kernel"], conf["stride"][i],
                        bool(conf["residual"][i]), kind)
    x = F.avg_pool2d(x, x.shape[2:])
    x = F.conv2d(x, sd["fcn_out.weight"], sd["fcn_out.bias"])
    return x.squeeze(-1)


# --------------------------------------------------------------------------------------
# RT-ST-GCN — models/rtstgcn/rtstgcn.py
# --------------------------------------------------------------------------------------


def causal_box_sum(x, K, S):
    """``x @ Toeplitz`` along the last axis (rtstgcn.py:366-379): y[..,c] = sum_{i<K//S} x[.., c - i*S].

    Restated as K//S shifted adds (the algorithmic cost, not O(L^2)).
    """
    y = torch.zeros_like(x)
    L = x.shape[-1]
    for i in range(K // S):
        s = i * S
        if s < L:
            y[..., s:] = y[..., s:] + x[..., : L - s]
    return y


def rt_offline_layer(x, A, sd, prefix, K, S, residual, normalization, importance=True):
    """OfflineLayer.forward (rtstgcn.py:343-389) with the Toeplitz it intends (self.toeplitz bug fixed)."""
    g = lambda k: sd[prefix + k]  # noqa: E731
    cin = x.shape[1]
    cout = g("conv.weight").shape[0] // A.shape[0]
    if not residual:
        res = 0
    elif cin == cout and S == 1:
        res = x
    else:
        r = F.conv2d(x, g("residual.0.weight"))  # no bias, no stride (rtstgcn.py:330)
        res = norm(normalization, r, g("residual.1.weight"), g("residual.1.bias"))
    Aeff = A * g("edge_importance") if importance else A
    N, _, L, V = x.shape
    P = A.shape[0]
    z = F.conv2d(x, g("conv.weight"), g("conv.bias"))            # (N, P*C, L, V)
    z = z.view(N, P, cout, L, V)                                   # split on dim 1 = partition-major
    z = torch.einsum("npclv,pvw->npclw", z, Aeff)                 # matmul with A (rtstgcn.py:364)
    z = z.sum(dim=1)                                               # sum over partitions (rtstgcn.py:381)
    z = causal_box_sum(z.permute(0, 1, 3, 2), K, S).permute(0, 1, 3, 2)
    h = torch.relu(norm(normalization, z, g("bn_relu.0.weight"), g("bn_relu.0.bias")))
    out = h + res
    return torch.relu(out) if residual else out


def rt_model_offline(x, sd, arch):
    """rt-st-gcn Model.forward (rtstgcn.py:137-157) with OfflineLayers."""
    conf = arch["rt-st-gcn"]
    kind = arch["normalization"]
    if kind == "LayerNorm":
        x = layernorm_cv(x, sd["norm_in.weight"], sd["norm_in.bias"])
    else:
        x = input_batchnorm(x, sd["norm_in.norm.weight"], sd["norm_in.norm.bias"])
    x = F.conv2d(x, sd["fcn_in.weight"], sd["fcn_in.bias"])
    for i in range(conf["layers"]):
        x = rt_offline_layer(x, sd["A"], sd, "st_gcn.%d." % i, conf["kernel"], conf["stride"][i],
                             bool(conf["residual"][i]), kind, conf["importance"])
    x = x.mean(dim=3, keepdim=True)                                # AvgPool2d((1,V))
    x = F.conv2d(x, sd["fcn_out.weight"], sd["fcn_out.bias"])
    return x.squeeze(-1)


class RtOnlineState:
    """Per-layer FIFO + accumulators of AggregateStgcn (rtstgcn.py:556-627), batch 1."""

    def __init__(self, cout, V, K, S):
        self.fifo_size = S * (K - 1) + 1                           # rtstgcn.py:477
        self.S = S
        self.fifo = torch.zeros(cout, self.fifo_size, V)
        self.acc = torch.zeros(cout, S, V)
        self.fi = 0
        self.ai = 0

    def push(self, z):
        """acc[ai] += z - fifo[fi]; out = acc[ai]; fifo[fi] = z (rtstgcn.py:611-625)."""
        self.acc[:, self.ai] = self.acc[:, self.ai] + z - self.fifo[:, self.fi]
        out = self.acc[:, self.ai].clone()
        self.fifo[:, self.fi] = z
        self.ai = (self.ai + 1) % self.S
        self.fi = (self.fi + 1) % self.fifo_size
        return out


def rt_model_online(frames, sd, arch):
    """Per-frame inference: _swap_layers_for_inference + eval_ + OnlineLayer.forward
    (rtstgcn.py:160-187, 522-553, 591-627).  ``frames`` is (1, C, L, V); returns (1, classes, L)."""
    conf = arch["rt-st-gcn"]
    kind = arch["normalization"]
    V = frames.shape[-1]
    A = sd["A"]
    P = A.shape[0]
    states = []
    for i in range(conf["layers"]):
        states.append(RtOnlineState(conf["out_ch"][i], V, conf["kernel"], conf["stride"][i]))
    outs = []
    for t in range(frames.shape[2]):
        x = frames[:, :, t:t + 1]
        if kind == "LayerNorm":
            x = layernorm_cv(x, sd["norm_in.weight"], sd["norm_in.bias"])
        else:
            x = input_batchnorm(x, sd["norm_in.norm.weight"], sd["norm_in.norm.bias"])
        x = F.conv2d(x, sd["fcn_in.weight"], sd["fcn_in.bias"])
        for i in range(conf["layers"]):
            pre = "st_gcn.%d." % i
            g = lambda k: sd[pre + k]  # noqa: E731
            cin, cout, S = conf["in_ch"][i], conf["out_ch"][i], conf["stride"][i]
            residual = bool(conf["residual"][i])
            if not residual:
                res = x * 0.0
            elif cin == cout and S == 1:
                res = x
            else:
                r = F.conv2d(x, g("residual.0.weight"))
                res = norm(kind, r, g("residual.1.weight"), g("residual.1.bias"))
            Aeff = A * g("edge_importance") if conf["importance"] else A   # eval_() fold
            z = F.conv2d(x, g("conv.weight"), g("conv.bias")).view(P, cout, V)
            z = torch.einsum("pcv,pvw->cw", z, Aeff)
            z = states[i].push(z).view(1, cout, 1, V)
            h = torch.relu(norm(kind, z, g("bn_relu.0.weight"), g("bn_relu.0.bias")))
            x = torch.relu(h + res) if residual else h + res
        x = x.mean(dim=3, keepdim=True)
        x = F.conv2d(x, sd["fcn_out.weight"], sd["fcn_out.bias"]).squeeze(-1)
        outs.append(x)
    return torch.cat(outs, dim=2)


# --------------------------------------------------------------------------------------
# AAGCN — models/aagcn/aagcn.py
# --------------------------------------------------------------------------------------


def agcn_layer(x, A, sd, prefix, kt, stride, residual, normalization, P):
    """AgcnLayer.forward (aagcn.py:139-150): softmax attention adjacency + StgcnLayer with A+B+C."""
    g = lambda k: sd[prefix + k]  # noqa: E731
    N, _, L, V = x.shape
    theta = F.conv2d(x, g("theta.weight"), g("theta.bias"))
    ce = theta.shape[1] // P
    theta = theta.view(N, P, ce * L, V).permute(0, 1, 3, 2)
    phi = F.conv2d(x, g("phi.weight"), g("phi.bias")).view(N, P, ce * L, V)
    C = torch.softmax(torch.matmul(theta, phi), dim=3)
    return stgcn_layer(x, A + g("B") + C, sd, prefix + "st_gcn.", kt, stride, residual, normalization)


def bones(x, A_raw_far):
    """Joint -> bone vectors (aagcn.py:63-68): x_bone[..., far(i)] = x[..., far(i)] - x[..., i]."""
    xb = torch.zeros_like(x)
    far = np.asarray(A_raw_far).astype(bool)
    for i in range(x.shape[-1]):
        idx = np.nonzero(far[i])[0]
        if len(idx):
            xb[:, :, :, idx] = x[:, :, :, idx] - x[:, :, :, i:i + 1]
    return xb


def aagcn_model(x, sd, arch, A_raw_far):
    """aa-gcn Model.forward (aagcn.py:60-95)."""
    conf = arch["aa-gcn"]
    kind = arch["normalization"]
    P = sd["A"].shape[0]
    ot = arch["output_type"]
    prob = {"logits": lambda t: t, "logsoftmax": lambda t: F.log_softmax(t, 1),
            "softmax": lambda t: F.softmax(t, 1)}[ot]
    xb = bones(x, A_raw_far)
    outs = []
    for s, xs in ((0, x), (1, xb)):
        pre = "streams.%d." % s
        if kind == "LayerNorm":
            xs = layernorm_cv(xs, sd[pre + "norm_in.weight"], sd[pre + "norm_in.bias"])
        else:
            xs = input_batchnorm(xs, sd[pre + "norm_in.norm.weight"], sd[pre + "norm_in.norm.bias"])
        xs = F.conv2d(xs, sd[pre + "fcn_in.weight"], sd[pre + "fcn_in.bias"])
        for i in range(conf["layers"]):
            xs = agcn_layer(xs, sd["A"], sd, pre + "gcn_networks.%d." % i, conf["kernel"], conf["stride"][i],
                            bool(conf["residual"][i]), kind, P)
        xs = F.avg_pool2d(xs, xs.shape[2:])
        xs = F.conv2d(xs, sd[pre + "fcn_out.weight"], sd[pre + "fcn_out.bias"])
        outs.append(xs.squeeze(-1))
    return prob(outs[1]) + prob(outs[0])


# --------------------------------------------------------------------------------------
# Loss — utils/loss.py:6-41 (output_type 'logits')
# --------------------------------------------------------------------------------------


def loss(i, logits, labels, class_dist, output_type="logits"):
    """Weighted CE + 0.15 * clamped temporal MSE (loss.py:8-41); output_type picks foo/bar (loss.py:10-18)."""
    w = 1 - class_dist / class_dist.sum()
    foo = {"logits": lambda x: x, "logsoftmax": lambda x: x, "softmax": torch.log}[output_type]
    bar = {"logits": lambda x: F.log_softmax(x, dim=1), "logsoftmax": torch.exp, "softmax": lambda x: x}[output_type]
    ce = F.cross_entropy(foo(logits if i == 0 else logits[:, :, 1:]), labels, weight=w)
    q = bar(logits)
    mse = 0.15 * torch.clamp((q[:, :, 1:] - q.detach()[:, :, :-1]) ** 2, 0, 16).mean()
    return ce, mse


def loss_shard(i, pred, labels, class_dist, prev, den, pairs, rank_first, output_type="logits"):
    """One data-parallel shard's share of loss.py:25-41 over the whole series: pred (1, C, n) this shard's
    frames, labels its labels (frame 0 dropped if i > 0 and rank_first), prev (C,) the frame before the
    shard or None, den = sum of class weights over the series' labels, pairs = series length - 1.  The
    shares of all shards sum to loss(i, series, ...); the MSE's left operand is detached (loss.py:37)."""
    w = 1 - class_dist / class_dist.sum()
    foo = {"logits": lambda x: x, "logsoftmax": lambda x: x, "softmax": torch.log}[output_type]
    bar = {"logits": lambda x: F.log_softmax(x, dim=1), "logsoftmax": torch.exp, "softmax": lambda x: x}[output_type]
    z = foo(pred if (i == 0 or not rank_first) else pred[:, :, 1:])
    ce = F.cross_entropy(z, labels, weight=w, reduction="sum") / den
    q = bar(pred)
    if prev is not None:
        q_prev = bar(prev.reshape(1, -1, 1).to(pred.dtype)).detach()
        qa = torch.cat([q_prev, q.detach()[:, :, :-1]], dim=2)
        qb = q
    else:
        qa, qb = q.detach()[:, :, :-1], q[:, :, 1:]
    mse = 0.15 * torch.clamp((qb - qa) ** 2, 0, 16).sum() / (pred.shape[1] * pairs)
    return ce, mse


def statistics(i, predictions, labels):
    """Top-1 / top-5 hits (statistics.py:5-16)."""
    p = predictions if i == 0 else predictions[:, :, 1:]
    _, top5 = torch.topk(p, k=5, dim=1)
    top1 = top5[:, 0, :]
    return top1, top5, int(torch.sum(top1 == labels)), int(torch.sum(top5 == labels[:, None])), labels.numel()


# --------------------------------------------------------------------------------------
# FLOP accounting used by bench.py
# --------------------------------------------------------------------------------------


def stgcn_layer_flops(N, T_in, V, cin, cout, P, kt, stride):
    t_out = math.ceil(T_in / stride)
    f = 2 * N * T_in * V * cin * P * cout + 2 * N * P * cout * T_in * V * V + 2 * N * t_out * V * cout * cout * kt
    if cin != cout or stride != 1:
        f += 2 * N * t_out * V * cin * cout
    return f

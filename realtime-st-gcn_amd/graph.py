"""Skeleton graph -> partitioned, normalised adjacency (host-side setup, numpy fp64).

Same construction as the reference's ``Graph`` (models/utils/graph.py:3-243): hop distances
(graph.py:182-205), spatial / distance / uniform partitioning (graph.py:108-170; 'uniform' is
all-zeros there, graph.py:134-135, and kept so), per-partition degree normalisation with the
alpha floor (graph.py:208-243) and the final transpose (graph.py:179) that makes row w of
``A[p]`` aggregate joint v in ``x @ A``.  The result is golden-pinned (tests/test_graph.py).
"""
from __future__ import annotations

import numpy as np

# PKU-MMD skeleton (25 joints, centre 20) — the graph of every BASELINE config.
PKU_MMD = {
    "num_node": 25,
    "edge": [[i, i] for i in range(25)] + [
        [0, 1], [1, 20], [2, 20], [3, 2], [4, 20], [5, 4], [6, 5], [7, 6], [8, 20], [9, 8], [10, 9], [11, 10],
        [12, 0], [13, 12], [14, 13], [15, 14], [16, 0], [17, 16], [18, 17], [19, 18], [21, 7], [22, 7], [23, 11],
        [24, 11]],
    "center": 20,
}


class Graph:
    """Partitioned skeleton adjacency.  Attributes mirror the reference: ``A`` (P,V,V) normalised
    and transposed, ``num_node``, ``edge``, ``center``, ``hop_dis``; ``get_adjacency_raw()``."""

    def __init__(self, num_node, edge, center, strategy="spatial", normalization="symmetric", max_hop=1,
                 dilation=1, alpha=0.001):
        self.num_node, self.edge, self.center = num_node, edge, center
        self.max_hop, self.dilation, self.alpha = max_hop, dilation, alpha
        self.hop_dis = self._hops()
        self._A = self.get_adjacency("spatial")
        A = self.get_adjacency(strategy)
        self.A = self._normalise(A, normalization == "symmetric")

    def _hops(self):
        V = self.num_node
        d = np.full((V, V), np.inf)
        e = np.asarray(self.edge, dtype=np.int64).reshape(-1, 2)
        self_loop = e[:, 0] == e[:, 1]
        d[e[self_loop, 0], e[self_loop, 0]] = 0
        d[e[~self_loop, 0], e[~self_loop, 1]] = 1
        d[e[~self_loop, 1], e[~self_loop, 0]] = 1
        for k in range(V):  # Floyd-Warshall, vectorised over (i, j)
            d = np.minimum(d, d[:, [k]] + d[[k], :])
        return d

    def get_adjacency_raw(self):
        return self._A

    def get_adjacency(self, strategy):
        V = self.num_node
        hops = list(range(0, self.max_hop + 1, self.dilation))
        reach = np.isin(self.hop_dis, hops).astype(np.float64)
        if strategy == "uniform":
            return np.zeros((1, V, V))
        if strategy == "distance":
            return np.stack([np.where(self.hop_dis == h, reach, 0.0) for h in hops])
        if strategy != "spatial":
            raise ValueError("Strategy Does Not Exist.")
        to_center = self.hop_dis[:, self.center]
        closer = to_center[None, :] < to_center[:, None]   # j nearer the centre than i
        same = to_center[None, :] == to_center[:, None]
        parts = []
        for h in hops:
            at_h = np.where(self.hop_dis == h, reach, 0.0)
            if h == 0:
                parts.append(np.where(same, at_h, 0.0))
            else:
                parts.append(np.where(closer, at_h, 0.0))
                parts.append(np.where(~closer & ~same, at_h, 0.0))
        return np.stack(parts)

    def _normalise(self, A, symmetric):
        out = np.empty_like(A)
        for p in range(A.shape[0]):
            with np.errstate(divide="ignore"):
                dl = np.power(A[p].sum(1) + self.alpha, -0.5 if symmetric else -1.0)
            dl[np.isinf(dl)] = 0
            out[p] = (dl[:, None] * A[p] * dl[None, :]) if symmetric else (A[p] * dl[None, :])
        return out.transpose(0, 2, 1)

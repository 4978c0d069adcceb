"""Synthetic workloads of BASELINE.md / SURVEY.md §8(d) (the reference has no benchmark data;
real datasets need network).

Chung-Lu power-law graph: p_i ∝ (i+1)^-alpha; E sources and E destinations drawn i.i.d.
from p (inverse-CDF sampling on a seeded CPU generator, so the graph is identical on every
machine), node ids relabelled by a random permutation to destroy locality; self-loops and
multi-edges kept (DGL allows both).
"""
import torch

from .graph import Graph

NAMED = {
    # name: (V, E, alpha)
    "S1": (500_000, 10_000_000, 0.8),      # 1-GPU kernel target
    "S2": (2_000_000, 40_000_000, 0.8),    # 1/2/4/8-GPU config 4
    "S1u": (500_000, 10_000_000, 0.0),     # uniform-degree control
    "arxiv": (169_343, 1_166_243, 0.8),    # ogbn-arxiv-shaped (config 3)
}


def powerlaw_edges(V, E, alpha=0.8, seed=0, chunk=1 << 24):
    g = torch.Generator().manual_seed(seed)
    p = (torch.arange(V, dtype=torch.float64) + 1.0).pow(-alpha)
    cdf = torch.cumsum(p, 0)
    cdf /= cdf[-1].clone()
    out = []
    for side in range(2):
        idx = torch.empty(E, dtype=torch.int64)
        for s in range(0, E, chunk):
            n = min(chunk, E - s)
            u = torch.rand(n, dtype=torch.float64, generator=g)
            idx[s:s + n] = torch.searchsorted(cdf, u, right=True).clamp_(max=V - 1)
        out.append(idx)
    relabel = torch.randperm(V, generator=g)
    return relabel[out[0]], relabel[out[1]]


def powerlaw_graph(V, E, alpha=0.8, seed=0):
    src, dst = powerlaw_edges(V, E, alpha, seed)
    return Graph(src, dst, V)


def named_graph(name, seed=0):
    V, E, alpha = NAMED[name]
    return powerlaw_graph(V, E, alpha, seed)

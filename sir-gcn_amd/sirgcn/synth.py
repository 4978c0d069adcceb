"""Synthetic workloads of BASELINE.md / SURVEY.md §8(d) (the reference has no benchmark data;
real datasets need network).

Chung-Lu power-law graph: p_i ∝ (i+1)^-alpha; E sources and E destinations drawn i.i.d.
from p (inverse-CDF sampling on a seeded CPU generator, so the graph is identical on every
machine), node ids relabelled by a random permutation to destroy locality; self-loops and
multi-edges kept (DGL allows both).
"""
import torch

from .graph import Graph, batch

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


def molecule_graph(n, rings, gen):
    """A molecule-shaped graph: a random tree over n atoms plus ``rings`` ring-closing bonds,
    every bond as two directed edges (OGB / benchmarking-GNNs molecules are bidirected)."""
    parent = [int(torch.randint(0, i, (1,), generator=gen)) for i in range(1, n)]
    u = list(range(1, n))
    v = parent
    for _ in range(rings if n > 4 else 0):
        a = int(torch.randint(0, n, (1,), generator=gen))
        b = int(torch.randint(0, n, (1,), generator=gen))
        if a != b:
            u.append(a)
            v.append(b)
    src = torch.tensor(u + v, dtype=torch.int64)
    dst = torch.tensor(v + u, dtype=torch.int64)
    return Graph(src, dst, n)


def molecule_batch(num_graphs, mean_nodes, seed=0, min_nodes=6, ring_closures=3):
    """``dgl.batch`` of molecule-shaped graphs with ~``mean_nodes`` atoms and ~``ring_closures``
    ring-closing bonds each: ZINC (~23.2 atoms, ~49.8 directed edges: ``molecule_batch(B, 23)``)
    and ogbg-molhiv (~25.5, ~55: ``molecule_batch(B, 25)``) statistics (the real
    datasets need network)."""
    gen = torch.Generator().manual_seed(seed)
    lo, hi = min_nodes, 2 * mean_nodes - min_nodes
    graphs = []
    for _ in range(num_graphs):
        n = int(torch.randint(lo, hi + 1, (1,), generator=gen))
        rings = int(torch.randint(0, 2 * ring_closures + 1, (1,), generator=gen))
        graphs.append(molecule_graph(n, rings, gen))
    return batch(graphs)


def dictionary_lookup_batch(n, num_graphs):
    """``synthetic-datasets/dictionary-lookup/data.py:27-31``: per graph 2n nodes, key nodes
    0..n-1, value nodes n..2n-1, the n^2 edges of the complete bipartite value->key graph
    (``itertools.product(val, key)`` order), batched ``num_graphs`` times."""
    key = torch.arange(n)
    val = torch.arange(n, 2 * n)
    src = val.repeat_interleave(n)
    dst = key.repeat(n)
    g = Graph(src, dst, 2 * n)
    return batch([g] * num_graphs)

"""TEST INFRASTRUCTURE: a CPU implementation of the three edge-pass entry points (same
signatures and item semantics as ``sirgcn._native``: a call covers exactly the edges of
``csr.items`` and writes only their rows; ``accumulate`` adds to the existing rows), built from
the oracle's sigma formulas, so the multi-rank partition / collective logic of ``sirgcn.dist``
(segmented forward, chunked backward) can be exercised with gloo on CPU.  Never used by the
product path."""
import torch

import oracle

ACT_NAMES = {0: "identity", 1: "relu", 2: "leaky", 3: "gelu", 4: "gelu_tanh"}


def _edges(csr):
    """(row, position) of every edge of the call's items, and the rows the items cover."""
    it = csr.items.long()
    if it.numel() == 0:
        z = torch.zeros(0, dtype=torch.int64)
        return z, z, z
    n = it[:, 2] - it[:, 1]
    pos = torch.repeat_interleave(it[:, 1], n) + (torch.arange(int(n.sum())) -
                                                    torch.repeat_interleave(torch.cumsum(n, 0) - n, n))
    return torch.repeat_interleave(it[:, 0], n), pos, torch.unique(it[:, 0])


def _store(out, full, rows, accumulate=False):
    if accumulate:
        out[rows] = out[rows] + full[rows]
    else:
        out[rows] = full[rows]


def edge_agg_fwd(csr, Q, K, norm_row, norm_col, agg, act, slope, S, partial, mask_out=None, accumulate=False):
    assert mask_out is None
    r, p, rows = _edges(csr)
    c = csr.col.long()[p]
    m = oracle.act_fwd(Q[r] + K[c], ACT_NAMES[act], slope)
    if agg == "sym":
        m = (norm_col[c] * norm_row[r]).unsqueeze(1) * m
    full = torch.zeros_like(S).index_add_(0, r, m)
    if agg == "mean":
        assert not accumulate
        rp = csr.rowptr.long()
        full = full / (rp[1:] - rp[:-1]).clamp(min=1).float().unsqueeze(1)
    _store(S, full, rows, accumulate)


def edge_agg_bwd_dst(csr, Q, K, G, norm_row, norm_col, agg, act, slope, dQ, Gm, partial, mask=None, drop=None):
    assert mask is None and drop is None
    r, p, rows = _edges(csr)
    c = csr.col.long()[p]
    rp = csr.rowptr.long()
    g = G / (rp[1:] - rp[:-1]).clamp(min=1).float().unsqueeze(1) if agg == "mean" else G
    if Gm is not None:
        Gm.copy_(g)
    t = g[r]
    if agg == "sym":
        t = t * (norm_col[c] * norm_row[r]).unsqueeze(1)
    dz = oracle.act_bwd(Q[r] + K[c], t, ACT_NAMES[act], slope)
    _store(dQ, torch.zeros_like(dQ).index_add_(0, r, dz), rows)


def edge_agg_bwd_src(csr_s, K, Q, Gd, norm_row, norm_col, agg, act, slope, dK, partial, mask=None, drop=None):
    assert mask is None and drop is None
    r, p, rows = _edges(csr_s)
    c = csr_s.col.long()[p]
    t = Gd[c]
    if agg == "sym":
        t = t * (norm_row[r] * norm_col[c]).unsqueeze(1)
    dz = oracle.act_bwd(Q[c] + K[r], t, ACT_NAMES[act], slope)
    _store(dK, torch.zeros_like(dK).index_add_(0, r, dz), rows)

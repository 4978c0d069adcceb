"""TEST INFRASTRUCTURE: a CPU implementation of the three edge-pass entry points (same
signatures as ``sirgcn._native``), built from the oracle's sigma formulas, so the multi-rank
partition / collective logic of ``sirgcn.dist`` can be exercised with gloo on CPU.  Never used
by the product path."""
import torch

import oracle

ACT_NAMES = {0: "identity", 1: "relu", 2: "leaky", 3: "gelu", 4: "gelu_tanh"}


def _rows(csr):
    rp = csr.rowptr.long()
    return torch.repeat_interleave(torch.arange(csr.n_rows), rp[1:] - rp[:-1]), csr.col.long()


def _deg(csr):
    rp = csr.rowptr.long()
    return (rp[1:] - rp[:-1]).clamp(min=1).float().unsqueeze(1)


def edge_agg_fwd(csr, Q, K, norm_row, norm_col, agg, act, slope, S, partial, mask_out=None):
    assert mask_out is None
    r, c = _rows(csr)
    m = oracle.act_fwd(Q[r] + K[c], ACT_NAMES[act], slope)
    if agg == "sym":
        m = (norm_col[c] * norm_row[r]).unsqueeze(1) * m
    out = torch.zeros_like(S).index_add_(0, r, m)
    if agg == "mean":
        out = out / _deg(csr)
    S.copy_(out)


def edge_agg_bwd_dst(csr, Q, K, G, norm_row, norm_col, agg, act, slope, dQ, Gm, partial, mask=None):
    assert mask is None
    r, c = _rows(csr)
    g = G / _deg(csr) if agg == "mean" else G
    if Gm is not None:
        Gm.copy_(g)
    t = g[r]
    if agg == "sym":
        t = t * (norm_col[c] * norm_row[r]).unsqueeze(1)
    dz = oracle.act_bwd(Q[r] + K[c], t, ACT_NAMES[act], slope)
    dQ.copy_(torch.zeros_like(dQ).index_add_(0, r, dz))


def edge_agg_bwd_src(csr_s, K, Q, Gd, norm_row, norm_col, agg, act, slope, dK, partial, mask=None):
    assert mask is None
    r, c = _rows(csr_s)
    t = Gd[c]
    if agg == "sym":
        t = t * (norm_row[r] * norm_col[c]).unsqueeze(1)
    dz = oracle.act_bwd(Q[c] + K[r], t, ACT_NAMES[act], slope)
    dK.copy_(torch.zeros_like(dK).index_add_(0, r, dz))

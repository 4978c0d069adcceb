"""Differentiable restatements of the reference layers, for chaining (TEST INFRASTRUCTURE ONLY).

``SIRConvRef`` restates ``models/conv.py:7-67`` and ``GraphNormRef`` ``models/norm.py:7-29`` as
torch modules with the reference's constructor signatures, so that ``sirgcn.stacks.SIRStack`` can
run the reference models' layer loops (configs 1/2/3/5) on them in fp32 (the reference's own
rounding) and fp64 (the truth the accuracy-aware parity checks measure against).  The dataflow
is the DGL edge-UDF path exactly as ``reference_cpu_step`` runs it (``index_select`` gathers,
elementwise UDF, ``index_add`` reduce, ``fn.mean`` = sum / clamp(deg, 1), ``fn.max`` first
arg-max wins) and autograd supplies the backward.  Works on any device (CPU, or torch on the
GPU for full-size checks — still only as the checker).

Pinning: ``tests/test_oracle_golden.py::test_oracle_modules_match_reference`` checks both
modules against the golden fixtures made by the reference's own ``conv.py`` / ``norm.py``.
"""
import torch
from torch import nn

from .sirconv_oracle import _MaxFirstWins


class SIRConvRef(nn.Module):
    """``conv.py:32-41`` parameters; ``conv.py:49-67`` forward (any sigma callable, any agg)."""

    def __init__(self, input_dim, hidden_dim, output_dim, activation, dropout=0, inner_bias=True,
                 outer_bias=True, agg_type='sum'):
        super().__init__()
        self.activation = activation
        self.dropout = nn.Dropout(dropout)
        self.linear_query = nn.Linear(input_dim, hidden_dim, bias=inner_bias)
        self.linear_key = nn.Linear(input_dim, hidden_dim, bias=False)
        self.linear_relation = nn.Linear(hidden_dim, output_dim, bias=outer_bias)
        self._agg_type = agg_type
        # conditioning (tests): qk_inject — a list of [V, 2H] value tensors, one consumed per forward,
        # whose VALUES replace Q, K while the gradients still flow through the projections
        # (straight-through); qk_record — a list that receives this forward's [Q | K] values
        self.qk_inject = None
        self.qk_record = None

    def forward(self, graph, feat):
        src, dst = (torch.as_tensor(t, dtype=torch.int64).to(feat.device) for t in graph.edges())
        V = int(graph.num_nodes())
        in_deg = torch.bincount(dst, minlength=V)
        out_deg = torch.bincount(src, minlength=V)
        # conv.py:51-57: norms are fp32 whatever the model dtype
        in_degs = in_deg.float().clamp(min=1)
        out_degs = out_deg.float().clamp(min=1)
        if self._agg_type == "sym":
            in_norm, out_norm = torch.pow(in_degs, -0.5), torch.pow(out_degs, -0.5)
        else:
            in_norm, out_norm = torch.ones_like(in_degs), torch.ones_like(out_degs)
        K = self.dropout(self.linear_key(feat))                       # conv.py:60
        Q = self.dropout(self.linear_query(feat))                     # conv.py:61
        H = Q.shape[1]
        if self.qk_inject:
            v = self.qk_inject.pop(0).to(device=Q.device, dtype=Q.dtype)
            Q = Q + (v[:, :H] - Q).detach()
            K = K + (v[:, H:] - K).detach()
        if self.qk_record is not None:
            self.qk_record.append(torch.cat([Q, K], 1).detach())
        a = self.activation(Q.index_select(0, dst) + K.index_select(0, src))   # conv.py:45
        if self._agg_type == "max":                                   # conv.py:46-47, DGL fn.max
            return _MaxFirstWins.apply(self.linear_relation(a), dst, V)
        m = (out_norm[src] * in_norm[dst]).unsqueeze(-1) * a          # conv.py:45 operand order
        S = torch.zeros((V, m.shape[1]), dtype=m.dtype, device=m.device).index_add(0, dst, m)
        if self._agg_type == "mean":                                  # fn.mean
            S = S / in_deg.clamp(min=1).to(S.dtype).unsqueeze(-1)
        return self.linear_relation(S)                                # conv.py:65


class GraphNormRef(nn.Module):
    """``norm.py:7-29`` (per-graph mean / variance of the mean_scale-shifted values)."""

    def __init__(self, normalized_shape, eps=1e-05, bias=True, mean_scale=True):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(normalized_shape))
        self.bias = nn.Parameter(torch.zeros(normalized_shape)) if bias else 0
        self.mean_scale = nn.Parameter(torch.ones(normalized_shape)) if mean_scale else 1

    def forward(self, graphs, feats):
        n = torch.as_tensor(graphs.batch_num_nodes(), dtype=torch.int64).to(feats.device)
        B = n.numel()
        gid = torch.repeat_interleave(torch.arange(B, device=feats.device), n)
        nf = n.to(feats.dtype).unsqueeze(1)
        mean = torch.zeros((B, feats.shape[1]), dtype=feats.dtype, device=feats.device).index_add(0, gid, feats) / nf
        demean = feats - mean[gid] * self.mean_scale
        var = torch.zeros_like(mean).index_add(0, gid, demean * demean) / nf
        std = torch.sqrt(var + self.eps)
        return self.weight * demean / std[gid] + self.bias

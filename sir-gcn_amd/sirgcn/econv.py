"""Drop-in ``SIREConv`` (SIR-GCN with edge features), briangodwinlim/SIR-GCN ``models/conv.py:70-134``.

    h_u^* = sum_{v in N(u)} W_R sigma(W_Q h_u + W_E h_{u,v} + W_K h_v)

Same constructor ``SIREConv(input_dim, edge_dim, hidden_dim, output_dim, activation, dropout=0,
inner_bias=True, outer_bias=True, agg_type='sum')`` (``conv.py:94``), attributes (``linear_edge``
has no bias, ``conv.py:99``; callers may swap it for an ``nn.Embedding``, ``zinc/model.py:12-15``)
and ``forward(graph, nfeat, efeat)`` (``conv.py:114``).

Runs on the edge-materialised native path (``sirgcn.generic``): ``z_e = (Q[v] + K[u]) + e_uv`` in
the reference's operand order (``conv.py:108``) with the node gathers done by
``sir_edge_gather_add``, the edge term ``e = dropout(linear_edge(efeat))`` permuted once into
destination-CSR order, sigma (any callable) by torch, then ``sir_segment_sum`` /
``sir_segment_max`` and their backward kernels.  No caller in the reference enables SIREConv
(it is commented out in every model), so this path is for API completeness, not a bench line.
"""
import torch
from torch import nn

from .generic import EdgeGatherAdd, EdgeMax, EdgeSum
from .graph import DEFAULT_CHUNK, get_plan


class SIREConv(nn.Module):
    def __init__(self, input_dim, edge_dim, hidden_dim, output_dim, activation, dropout=0, inner_bias=True,
                 outer_bias=True, agg_type='sum'):
        super().__init__()
        if agg_type not in ("sum", "mean", "sym", "max"):
            raise AttributeError(f"module 'dgl.function' has no attribute '{agg_type}'")
        self.activation = activation
        self.dropout = nn.Dropout(dropout)
        self.linear_query = nn.Linear(input_dim, hidden_dim, bias=inner_bias)
        self.linear_key = nn.Linear(input_dim, hidden_dim, bias=False)
        self.linear_edge = nn.Linear(edge_dim, hidden_dim, bias=False)
        self.linear_relation = nn.Linear(hidden_dim, output_dim, bias=outer_bias)
        self._agg_type = agg_type
        self.chunk = DEFAULT_CHUNK

    def forward(self, graph, nfeat, efeat):
        if isinstance(nfeat, tuple):         # expand_as_pair (conv.py:126)
            nfeat_key, nfeat_query = nfeat
        else:
            nfeat_key = nfeat_query = nfeat
        if nfeat_query.device.type != "cuda":
            raise RuntimeError("SIREConv native path needs a ROCm GPU tensor (no CPU fallback)")
        plan = get_plan(graph, nfeat_query.device, self.chunk)
        if plan.num_nodes != nfeat_query.shape[0]:
            raise ValueError(f"nfeat has {nfeat_query.shape[0]} rows, graph has {plan.num_nodes} nodes")
        if efeat.shape[0] != plan.num_edges:
            raise ValueError(f"efeat has {efeat.shape[0]} rows, graph has {plan.num_edges} edges")
        H = self.linear_query.out_features
        K = self.dropout(self.linear_key(nfeat_key))                     # conv.py:127
        Q = self.dropout(self.linear_query(nfeat_query))                 # conv.py:128
        Ee = self.dropout(self.linear_edge(efeat))                       # conv.py:129
        Z = EdgeGatherAdd.apply(torch.cat([Q, K], 1), plan, H)           # eq[v] + ek[u], dst-CSR order
        Z = Z + Ee.index_select(0, plan.dst.eid).to(Z.dtype)             # (...) + e_uv (conv.py:108)
        A = self.activation(Z)
        if self._agg_type == "max":
            return EdgeMax.apply(self.linear_relation(A), plan)           # conv.py:110, no post-projection
        S = EdgeSum.apply(A, plan, self._agg_type)                       # conv.py:108 norms, 131 update_all
        return self.linear_relation(S)                                   # conv.py:133

    def extra_repr(self):
        return f"agg_type={self._agg_type!r}"

"""Edge-materialised SIRConv path: ``agg_type='max'`` and arbitrary ``activation`` callables.

Sparse steps compute in fp32 (results are returned in the caller's dtype).  The reference
runs every variant through DGL's edge-UDF path (``conv.py:43-47,63``): gather
``eq[v] + ek[u]`` per edge, apply the UDF (sigma, and for ``max`` also ``linear_relation``), then
reduce.  The fused kernels (``conv.py`` here) cover elementwise sigma with sum/mean/sym.  For the
rest this module keeps the UDF dataflow but runs every sparse step natively (``sir_edge_gather_add``,
``sir_segment_sum``, ``sir_edge_broadcast``, ``sir_segment_max``, ``sir_segment_max_bwd``); the
UDF itself (any torch callable, e.g. DictionaryLookup's ``Sequential(ReLU, Linear, ReLU)``,
``dictionary-lookup/model.py:17``, or ``linear_relation`` for ``max``) runs as torch ops on
``[E, F]`` edge rows in destination-CSR order, with autograd.

``max`` follows DGL's ``SpMMCmpCsr``: elementwise max over in-edges, the gradient goes to the
FIRST arg-max edge (ties keep the earlier edge), rows without in-edges output 0.
"""
import torch

from . import _native


def _ws(n_slots, F, device, dtype=torch.float32):
    return torch.empty((max(n_slots, 1) * F,), device=device, dtype=dtype) if n_slots else None


class EdgeGatherAdd(torch.autograd.Function):
    """Z[e] = Q[dst(e)] + K[src(e)] for QK = [Q | K] ([V, 2H]); edges in dst-CSR order."""

    @staticmethod
    def forward(ctx, QK, plan, H):
        ctx.in_dtype = QK.dtype
        QK = QK.contiguous().float()
        E = plan.dst.col.numel()
        Z = torch.empty((E, H), device=QK.device, dtype=torch.float32)
        _native.edge_gather_add(plan.dst, QK[:, :H], QK[:, H:], Z)
        ctx.plan, ctx.H, ctx.V = plan, H, QK.shape[0]
        return Z.to(ctx.in_dtype)

    @staticmethod
    def backward(ctx, dZ):
        plan, H = ctx.plan, ctx.H
        dZ = dZ.contiguous().float()
        dQK = torch.empty((ctx.V, 2 * H), device=dZ.device, dtype=torch.float32)
        n_slots = max(plan.dst.n_slots, plan.src.n_slots)
        partial = _ws(n_slots, H, dZ.device)
        _native.segment_sum(plan.dst, dZ, dQK[:, :H], partial=partial)                   # dQ: index_add by dst
        _native.segment_sum(plan.src, dZ, dQK[:, H:], perm=plan.src.perm, partial=partial)  # dK: by src
        return dQK.to(ctx.in_dtype), None, None


class EdgeSum(torch.autograd.Function):
    """S[v] = sum_{e->v} (out_norm[u] * in_norm[v]) * M[e]  (sym), or plain sum / mean."""

    @staticmethod
    def forward(ctx, M, plan, agg):
        ctx.in_dtype = M.dtype
        M = M.contiguous().float()
        F = M.shape[1]
        in_norm, out_norm = plan.norms(agg)
        S = torch.empty((plan.dst.n_rows, F), device=M.device, dtype=torch.float32)
        _native.segment_sum(plan.dst, M, S, in_norm, out_norm, agg == "mean",
                            partial=_ws(plan.dst.n_slots, F, M.device))
        ctx.plan, ctx.agg, ctx.E = plan, agg, M.shape[0]
        return S.to(ctx.in_dtype)

    @staticmethod
    def backward(ctx, dS):
        plan, agg = ctx.plan, ctx.agg
        dS = dS.contiguous().float()
        in_norm, out_norm = plan.norms(agg)
        dM = torch.empty((ctx.E, dS.shape[1]), device=dS.device, dtype=torch.float32)
        _native.edge_broadcast(plan.dst, dS, dM, in_norm, out_norm, agg == "mean")
        return dM.to(ctx.in_dtype), None, None


class EdgeMax(torch.autograd.Function):
    """Y[v] = max_{e->v} M[e] (DGL fn.max: first arg-max gets the gradient, empty rows -> 0)."""

    @staticmethod
    def forward(ctx, M, plan):
        ctx.in_dtype = M.dtype
        M = M.contiguous().float()
        F = M.shape[1]
        V = plan.dst.n_rows
        Y = torch.empty((V, F), device=M.device, dtype=torch.float32)
        arg = torch.empty((V, F), device=M.device, dtype=torch.int32)
        n = plan.dst.n_slots
        _native.segment_max(plan.dst, M, Y, arg, _ws(n, F, M.device), _ws(n, F, M.device, torch.int32))
        ctx.save_for_backward(arg)
        ctx.plan, ctx.E = plan, M.shape[0]
        return Y.to(ctx.in_dtype)

    @staticmethod
    def backward(ctx, dY):
        (arg,) = ctx.saved_tensors
        dY = dY.contiguous().float()
        dM = torch.empty((ctx.E, dY.shape[1]), device=dY.device, dtype=torch.float32)
        _native.segment_max_bwd(ctx.plan.dst, arg, dY, dM)
        return dM.to(ctx.in_dtype), None


def generic_forward(conv, plan, feat_key, feat_query):
    """``conv.py:49-67`` through the edge-materialised path (``conv`` is a sirgcn.SIRConv)."""
    H = conv.linear_query.out_features
    QK = conv._project(feat_key, feat_query)
    Z = EdgeGatherAdd.apply(QK, plan, H)
    A = conv.activation(Z)                                   # any callable, autograd through torch
    if conv._agg_type == "max":
        M = conv._relation(A)                                # conv.py:47 per-edge W_R
        return EdgeMax.apply(M, plan)                        # conv.py:65: no post-projection for max
    S = EdgeSum.apply(A, plan, conv._agg_type)
    return conv._relation(S)

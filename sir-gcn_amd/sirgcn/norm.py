"""Fused GraphNorm on MI355X — drop-in for the reference ``models/norm.py:7-29`` ``GraphNorm``.

Same constructor ``GraphNorm(normalized_shape, eps=1e-05, bias=True, mean_scale=True)``, same
parameters (``weight``, ``bias`` (or the int 0), ``mean_scale`` (or the int 1)) and
``forward(graphs, feats)`` over a batched graph (``graphs.batch_num_nodes()``; a DGLGraph or
``sirgcn.graph.batch([...])``).  Per graph: mean / variance of the mean_scale-shifted values,
exactly as the reference (the variance is taken of ``feats - mean * mean_scale``).  One native
kernel per direction (``sir_graph_norm_fwd`` / ``sir_graph_norm_bwd``) replaces the reference's
~8 torch kernels (scatter_add x2, repeat_interleave x2, elementwise).
"""
import torch
from torch import nn

from . import _native
from .graph import node_offsets


class GraphNormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, weight, bias, mean_scale, off, eps):
        if X.device.type != "cuda":
            raise RuntimeError("sirgcn.GraphNorm needs a ROCm GPU tensor (no CPU fallback)")
        X = X.contiguous().float()
        B = off.numel() - 1
        F = X.shape[1]
        Y = torch.empty_like(X)
        mean = torch.empty((B, F), device=X.device, dtype=torch.float32)
        std = torch.empty_like(mean)
        w = weight.contiguous().float()
        b = bias.contiguous().float() if bias is not None else None
        ms = mean_scale.contiguous().float() if mean_scale is not None else None
        _native.graph_norm_fwd(off, X, w, b, ms, eps, Y, mean, std)
        ctx.save_for_backward(X, w, ms if ms is not None else w, mean, std, off)
        ctx.has_b, ctx.has_ms = bias is not None, mean_scale is not None
        return Y

    @staticmethod
    def backward(ctx, dY):
        X, w, ms, mean, std, off = ctx.saved_tensors
        ms = ms if ctx.has_ms else None
        dY = dY.contiguous().float()
        dX = torch.empty_like(X)
        # the per-graph partials of dw, db (and dms) as slabs of one [n, B, F] buffer, reduced over
        # the graphs by ONE launch (molecule batches are launch-bound: three column sums were six)
        parts = torch.empty((3 if ms is not None else 2,) + tuple(mean.shape), device=X.device, dtype=torch.float32)
        _native.graph_norm_bwd(off, X, dY, w, ms, mean, std, dX, parts[0], parts[2] if ms is not None else None,
                               parts[1])
        sums = parts.sum(1)
        dw = sums[0]
        db = sums[1] if ctx.has_b else None
        dms = sums[2] if ms is not None else None
        return dX, dw, db, dms, None, None


class GraphNorm(nn.Module):
    """``models/norm.py:7-29`` GraphNorm, fused (see module docstring)."""

    def __init__(self, normalized_shape, eps=1e-05, bias=True, mean_scale=True):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(normalized_shape))
        self.bias = nn.Parameter(torch.zeros(normalized_shape)) if bias else 0
        self.mean_scale = nn.Parameter(torch.ones(normalized_shape)) if mean_scale else 1

    def forward(self, graphs, feats):
        if feats.dim() != 2:
            raise ValueError("GraphNorm expects [num_nodes, features]")
        off = node_offsets(graphs, feats.device)
        b = self.bias if isinstance(self.bias, torch.Tensor) else None
        ms = self.mean_scale if isinstance(self.mean_scale, torch.Tensor) else None
        return GraphNormFunction.apply(feats, self.weight, b, ms, off, float(self.eps))

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


class GraphNormActFunction(torch.autograd.Function):
    """act(GraphNorm(X)) + R in one kernel per direction (``sir_graph_norm_act_fwd`` / ``_bwd``):
    the stack loop's ``norm -> activation -> + resid`` (ogbn-arxiv/model.py:65-73,
    ogbg-molhiv/model.py:76-84; R = None: zinc/model.py:54-55).  The same ops as the three torch
    calls, so the same bits; R's gradient is the incoming gradient itself."""

    @staticmethod
    def forward(ctx, X, weight, bias, mean_scale, off, eps, act, slope, R):
        X = X.contiguous().float()
        B = off.numel() - 1
        F = X.shape[1]
        Y = torch.empty_like(X)
        mean = torch.empty((B, F), device=X.device, dtype=torch.float32)
        std = torch.empty_like(mean)
        w = weight.contiguous().float()
        b = bias.contiguous().float() if bias is not None else None
        ms = mean_scale.contiguous().float() if mean_scale is not None else None
        Rc = R.contiguous() if R is not None else None
        _native.graph_norm_act_fwd(off, X, w, b, ms, eps, act, slope, Rc, Y, mean, std)
        ctx.save_for_backward(X, w, b if b is not None else w, ms if ms is not None else w, mean, std, off)
        ctx.has_b, ctx.has_ms, ctx.has_r = bias is not None, mean_scale is not None, R is not None
        ctx.act, ctx.slope = act, slope
        return Y

    @staticmethod
    def backward(ctx, dY):
        X, w, b, ms, mean, std, off = ctx.saved_tensors
        b = b if ctx.has_b else None
        ms = ms if ctx.has_ms else None
        dY = dY.contiguous().float()
        dX = torch.empty_like(X)
        parts = torch.empty((3 if ms is not None else 2,) + tuple(mean.shape), device=X.device, dtype=torch.float32)
        _native.graph_norm_act_bwd(off, X, dY, w, b, ms, mean, std, ctx.act, ctx.slope, dX, parts[0],
                                   parts[2] if ms is not None else None, parts[1])
        sums = parts.sum(1)
        return (dX, sums[0], sums[1] if ctx.has_b else None, sums[2] if ms is not None else None, None, None, None,
                None, dY if ctx.has_r else None)


def _act_code(m):
    """(code, slope) of an activation module the fused kernel applies, else None."""
    if isinstance(m, nn.ReLU):
        return _native.ACT_RELU, 0.0
    if isinstance(m, nn.LeakyReLU):
        return _native.ACT_LEAKY, float(m.negative_slope)
    if isinstance(m, nn.Identity):
        return _native.ACT_IDENTITY, 0.0
    return None


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

    def forward_act(self, graphs, feats, activation, resid=None):
        """``activation(self(graphs, feats)) + resid`` (resid None: no add) in one kernel per
        direction, or None when the activation / operands are not the fused kernel's, or a hook
        waits on either module's call (the caller then runs the three steps itself)."""
        code = _act_code(activation)
        hooked = any(len(h) for m in (self, activation) for h in (m._forward_pre_hooks, m._forward_hooks,
                                                                 m._backward_hooks, m._backward_pre_hooks))
        if (code is None or hooked or feats.dim() != 2 or not feats.is_cuda
                or (resid is not None and (resid.dtype != torch.float32 or resid.shape != feats.shape))):
            return None
        off = node_offsets(graphs, feats.device)
        b = self.bias if isinstance(self.bias, torch.Tensor) else None
        ms = self.mean_scale if isinstance(self.mean_scale, torch.Tensor) else None
        return GraphNormActFunction.apply(feats, self.weight, b, ms, off, float(self.eps), code[0], code[1], resid)

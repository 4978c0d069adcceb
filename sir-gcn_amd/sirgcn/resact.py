"""The stack loop's residual + activation around a SIRConv layer without a norm, one native pass
per direction (``sir_resid_act_fwd`` / ``_bwd``):

* zinc order (``zinc/model.py:53-56``): ``h = act(conv(g, h) + h)``;
* arxiv order without a norm (``ogbn-arxiv/model.py:65-73``): ``h = act(conv(g, h)) + h``.

Bit-identical to torch's separate add / activation kernels and their autograd (including the
autocast dtypes: a 16-bit conv output, an fp32 residual); replaces two kernels forward and two or
three backward (the 16-bit gradient cast included).

Chained layers (:class:`GradLink`): layer i's output h is both the next layer's conv input and its
residual, so autograd would add the two gradients of h in a pass of its own before layer i's backward
reads them.  With a link the next layer's pass hands its residual gradient over instead of returning
it, and layer i's backward adds it while reading the conv input's gradient (``D2`` of
``sir_resid_act_bwd``; arxiv order: the sum is also written once, as layer i's own residual gradient):
the same sum (a + b == b + a), one launch and one or two [V, H] passes fewer per layer.
"""
import torch
from torch import nn

from . import _native


def act_code(m):
    """(code, slope) of an activation module the native pass applies, else None."""
    if isinstance(m, nn.ReLU):
        return _native.ACT_RELU, 0.0
    if isinstance(m, nn.LeakyReLU):
        return _native.ACT_LEAKY, float(m.negative_slope)
    if isinstance(m, nn.Identity):
        return _native.ACT_IDENTITY, 0.0
    return None


def _ok(t, dtypes):
    return (t.is_cuda and t.dtype in dtypes and t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 4 == 0
            and t.data_ptr() % (16 if t.dtype == torch.float32 else 8) == 0)


class GradLink:
    """Hands one gradient from a layer's backward to the backward of the layer whose output it belongs
    to (see the module docstring).  Created per forward, so a value never outlives its graph."""
    __slots__ = ("grad",)

    def __init__(self):
        self.grad = None

    def put(self, g):
        self.grad = g

    def take(self):
        g, self.grad = self.grad, None
        return g


class ResidActFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Y, R, act, slope, order, r_link=None, out_link=None):
        # r_link: R is the output of a linked layer — put dR there instead of returning it;
        # out_link: this output's residual gradient from the next layer arrives there
        out = torch.empty(Y.shape, device=Y.device, dtype=torch.float32)
        _native.resid_act_fwd(Y, R, act, slope, order, out)
        ctx.save_for_backward(Y, R if order == 0 else None)
        ctx.act, ctx.slope, ctx.order = act, slope, order
        ctx.r_link, ctx.out_link = r_link, out_link
        return out

    @staticmethod
    def backward(ctx, D):
        Y, R = ctx.saved_tensors
        D = D.contiguous()
        dY = torch.empty_like(Y)
        if ctx.order == 0:
            D2 = ctx.out_link.take() if ctx.out_link is not None else None
            dR = torch.empty(Y.shape, device=Y.device, dtype=torch.float32)
            _native.resid_act_bwd(D, Y, R, ctx.act, ctx.slope, 0, dY, dR, D2=D2)
            if ctx.r_link is not None and ctx.needs_input_grad[1]:
                ctx.r_link.put(dR)
                dR = None
            return dY, dR, None, None, None, None, None
        D2 = ctx.out_link.take() if ctx.out_link is not None else None
        if D2 is not None:              # R's gradient is dout: the sum D + D2, formed by the pass
            dR = torch.empty(Y.shape, device=Y.device, dtype=torch.float32)
            _native.resid_act_bwd(D, Y, None, ctx.act, ctx.slope, 1, dY, dR, D2=D2)
        else:
            _native.resid_act_bwd(D, Y, None, ctx.act, ctx.slope, 1, dY)
            dR = D
        if ctx.r_link is not None and ctx.needs_input_grad[1]:
            ctx.r_link.put(dR)
            dR = None
        return dY, dR, None, None, None, None, None


def resid_act(y, resid, activation, order, r_link=None, out_link=None):
    """``activation(y + resid)`` (order "zinc") or ``activation(y) + resid`` ("arxiv") in one pass,
    or None when the activation / operands are not the native pass's (or a hook waits on the
    activation's call): the caller then runs the torch ops itself.  ``r_link`` / ``out_link``
    (:class:`GradLink`): ``resid`` is the output of the layer that holds ``r_link`` as
    its ``out_link`` — the residual gradient goes there instead of through autograd; ``out_link``
    receives the next layer's."""
    code = act_code(activation)
    hooked = any(len(h) for h in (activation._forward_pre_hooks, activation._forward_hooks,
                                  activation._backward_hooks, activation._backward_pre_hooks))
    if (code is None or hooked or order not in ("zinc", "arxiv") or y.shape != resid.shape or y.dim() != 2
            or y.shape[1] % 4 != 0 or not _ok(y, (torch.float32, torch.bfloat16, torch.float16))
            or not _ok(resid, (torch.float32,))):
        return None
    return ResidActFunction.apply(y, resid, code[0], code[1], 0 if order == "zinc" else 1, r_link, out_link)

"""Multi-layer SIRConv stacks: the layer loops of the reference's models, i.e. the callers of the
hot path for BASELINE configs 1, 2, 3 and 5.

The reference models wrap SIRConv in embeddings, readouts and pooling (out of scope);
what reaches the hot path is their per-layer loop, restated here with the conv / norm classes as
parameters so that the SAME loop runs on the reference's own ``models/conv.py`` / ``models/norm.py``
(``tests/golden/make_golden.py`` builds the stack fixtures that way) and on this package's
MI355X modules (tests, ``bench.py --workload``):

* ``order="arxiv"`` — ``ogbn-arxiv/model.py:65-73`` and ``ogbg-molhiv/model.py:76-84``:
  ``resid = h; h = conv(g, h); h = norm(g, h); h = act(h); h = h + resid``;
* ``order="zinc"`` — ``zinc/model.py:50-56`` (identity residual): ``h = conv(g, h) + h;
  h = norm(g, h); h = act(h)``;
* ``order="plain"`` — ``dictionary-lookup/model.py:30-32``: ``h = conv(g, h)`` (the
  ``Sequential`` sigma lives inside the conv).

``norm_cls`` (e.g. GraphNorm, ``models/norm.py:7-29``) is called as ``norm(graph, feats)``.
"""
from torch import nn


def _resid_act(y, resid, activation, order, r_link=None, out_link=None):
    """sirgcn.resact.resid_act for GPU tensors (imported lazily: the stack also runs the reference's
    own modules on the CPU, where it returns None)."""
    if not (getattr(y, "is_cuda", False) and getattr(resid, "is_cuda", False)):
        return None
    from .resact import resid_act
    return resid_act(y, resid, activation, order, r_link, out_link)


def _new_link():
    from .resact import GradLink
    return GradLink()


class SIRStack(nn.Module):
    # the fused residual pass (no norm): each layer's residual gradient handed to the previous layer's
    # backward (sirgcn.resact.GradLink) instead of an autograd add.  The parameters' and the
    # stack input's gradients are the same bits either way; a hook on (or torch.autograd.grad of) an
    # intermediate layer output sees only its conv-input part — set False for that.
    link_residual_grads = True

    def __init__(self, conv_cls, hidden, num_layers, activation, agg_type="sum", order="arxiv",
                 norm_cls=None, conv_activation=None, feat_dropout=0):
        super().__init__()
        if order not in ("arxiv", "zinc", "plain"):
            raise ValueError(order)
        self.order = order
        self.activation = activation
        sigma = conv_activation if conv_activation is not None else activation
        # feat_dropout: the conv's own Dropout on Q and K, passed positionally as the reference's
        # models do (ogbn-arxiv/model.py:57, ogbg-molhiv/model.py:66)
        self.convs = nn.ModuleList([conv_cls(hidden, hidden, hidden, sigma, feat_dropout, agg_type=agg_type)
                                    for _ in range(num_layers)])
        self.norms = nn.ModuleList([norm_cls(hidden) for _ in range(num_layers)]) if norm_cls else None

    def forward(self, graph, feats):
        if self.training and getattr(feats, "is_cuda", False):
            # the dropout seeds of every layer in ONE device draw (sirgcn SIRConv's step_seed): one
            # RNG launch per step instead of one per layer (small batches are launch-bound)
            drawing = [c for c in self.convs if hasattr(c, "step_seed") and c.dropout.p > 0]
            if drawing:
                import torch
                seeds = torch.randint(0, 2 ** 62, (len(drawing),), device=feats.device, dtype=torch.int64)
                for j, c in enumerate(drawing):
                    c.step_seed = seeds[j:j + 1]
        link = None          # the GradLink of feats when a fused residual pass produced it
        for i, conv in enumerate(self.convs):
            if self.order == "plain":
                feats = conv(graph, feats)
                continue
            resid = feats
            feats = conv(graph, feats)
            if self.norms is None:
                # + resid and the activation in one pass when the operands allow (sirgcn.resact);
                # the residual gradient of each layer's input handed to the layer that produced it
                # (resact.GradLink) instead of an autograd add
                out_link = _new_link() if self.link_residual_grads and getattr(feats, "is_cuda", False) else None
                fused = _resid_act(feats, resid, self.activation, self.order, link, out_link)
                if fused is not None:
                    feats = fused
                    link = out_link
                    continue
            link = None
            if self.order == "zinc":
                feats = feats + resid
            if self.norms is not None:
                # norm -> act (-> + resid) as one op when the norm offers it (sirgcn.GraphNorm:
                # one kernel per direction; None: not for this activation / these operands)
                fuse = getattr(self.norms[i], "forward_act", None)
                out = fuse(graph, feats, self.activation, resid if self.order == "arxiv" else None) if fuse else None
                if out is not None:
                    feats = out
                    continue
                feats = self.norms[i](graph, feats)
            feats = self.activation(feats)
            if self.order == "arxiv":
                feats = feats + resid
        return feats

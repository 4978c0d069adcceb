"""Test-only DGL-semantics shim (fixture generation in the build container ONLY).

DGL 2.1.0 (`requirements.txt:1` of the reference) is not installed and not vendored.
This shim restates the few pieces of DGL's published behaviour that the reference's
`models/conv.py` touches, so that the reference's OWN, unmodified `SIRConv` can be
executed here to produce golden vectors (`tests/golden/make_golden.py`).

Restated DGL 2.1.0 behaviour:
  * ``DGLGraph.update_all(udf, builtin_reduce)`` -> ``core.message_passing``:
    the edge UDF sees ``edges.src[k] = ndata[k][src]``, ``edges.dst[k] = ndata[k][dst]``
    (``index_select`` gathers in edge-id order); the builtin reducer is a GSpMM
    ``copy_e`` over the in-edge CSC.  CPU ``SpMMSumCsr`` accumulates each destination
    row sequentially in CSC order (ascending edge id, stable counting sort), starting
    from zero; ``index_add_`` over edge-id order yields the same per-row order.
  * ``fn.mean``  = sum / clamp(in_degree, 1) cast to the message dtype
    (``dgl/ops/spmm.py`` gspmm, reduce_op == 'mean').
  * ``fn.max``   = elementwise max over in-edges; 0 for isolated destinations.
    DGL sends the max gradient to the FIRST arg-max edge; this shim uses torch
    ``scatter_reduce('amax')`` whose backward splits ties -> max-tie gradients are
    parity-unpinned (documented in DESIGN.md).
  * ``expand_as_pair(x, g)`` returns ``(x, x)`` for a non-block graph.
  * ``dgl.batch`` concatenates node/edge ids with offsets and records ``batch_num_nodes``;
    ``dgl.broadcast_nodes(g, feat)`` repeats row b of ``feat`` for every node of graph b
    (used by ``models/norm.py:17`` GraphNorm).

This package is put on ``sys.path`` only by ``make_golden.py``; nothing on the product
path, the GPU box or the test-suite imports it.
"""
import contextlib

import torch

from . import function  # noqa: F401
from . import utils  # noqa: F401


class _Frame(dict):
    pass


class _LazyGather:
    """edges.src / edges.dst view: gathers rows of node data by an index on access."""

    def __init__(self, data, index):
        self._data = data
        self._index = index

    def __getitem__(self, key):
        return torch.index_select(self._data[key], 0, self._index)


class EdgeBatch:
    def __init__(self, ndata, edata, src, dst):
        self.src = _LazyGather(ndata, src)
        self.dst = _LazyGather(ndata, dst)
        self.data = edata


class DGLGraph:
    def __init__(self, src, dst, num_nodes, batch_num_nodes=None):
        self._src = torch.as_tensor(src, dtype=torch.int64)
        self._dst = torch.as_tensor(dst, dtype=torch.int64)
        self._n = int(num_nodes)
        self._bnn = (torch.tensor([self._n], dtype=torch.int64) if batch_num_nodes is None
                     else torch.as_tensor(batch_num_nodes, dtype=torch.int64))
        self.ndata = _Frame()
        self.edata = _Frame()

    # --- batching (dgl.batch semantics: node ids concatenated with offsets) -----------
    def batch_num_nodes(self):
        return self._bnn

    @property
    def batch_size(self):
        return int(self._bnn.numel())

    # --- structure ---------------------------------------------------------------
    def num_nodes(self):
        return self._n

    def num_edges(self):
        return int(self._src.numel())

    @property
    def device(self):
        return self._src.device

    def in_degrees(self):
        return torch.bincount(self._dst, minlength=self._n)

    def out_degrees(self):
        return torch.bincount(self._src, minlength=self._n)

    def edges(self):
        return self._src, self._dst

    @contextlib.contextmanager
    def local_scope(self):
        saved_n, saved_e = dict(self.ndata), dict(self.edata)
        try:
            yield
        finally:
            self.ndata = _Frame(saved_n)
            self.edata = _Frame(saved_e)

    # --- message passing -----------------------------------------------------------
    def update_all(self, message_func, reduce_func):
        eb = EdgeBatch(self.ndata, self.edata, self._src, self._dst)
        msg = message_func(eb)[reduce_func.msg_field]
        n = self._n
        out_shape = (n,) + tuple(msg.shape[1:])
        if reduce_func.name in ("sum", "mean"):
            out = torch.zeros(out_shape, dtype=msg.dtype, device=msg.device).index_add(0, self._dst, msg)
            if reduce_func.name == "mean":
                deg = self.in_degrees().clamp(1, max(self.num_edges(), 1)).to(out.dtype)
                out = out / deg.reshape((n,) + (1,) * (out.dim() - 1))
        elif reduce_func.name == "max":
            idx = self._dst.reshape((-1,) + (1,) * (msg.dim() - 1)).expand_as(msg)
            out = torch.zeros(out_shape, dtype=msg.dtype, device=msg.device).scatter_reduce(
                0, idx, msg, reduce="amax", include_self=False)
        else:
            raise NotImplementedError(reduce_func.name)
        self.ndata[reduce_func.out_field] = out


def batch(graphs):
    offs, src, dst, bnn = 0, [], [], []
    for g in graphs:
        src.append(g._src + offs)
        dst.append(g._dst + offs)
        bnn.append(g._n)
        offs += g._n
    return DGLGraph(torch.cat(src), torch.cat(dst), offs, torch.tensor(bnn, dtype=torch.int64))


def broadcast_nodes(graph, feat):
    """dgl.broadcast_nodes: row b of ``feat`` repeated for every node of graph b."""
    return torch.repeat_interleave(feat, graph.batch_num_nodes(), dim=0)


def graph(data, num_nodes=None):
    src, dst = data
    src = torch.as_tensor(src, dtype=torch.int64)
    dst = torch.as_tensor(dst, dtype=torch.int64)
    if num_nodes is None:
        num_nodes = int(max(src.max().item(), dst.max().item()) + 1) if src.numel() else 0
    return DGLGraph(src, dst, num_nodes)

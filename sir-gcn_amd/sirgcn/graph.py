"""Graph container and the per-graph work plans the edge kernels consume.

The reference hands ``SIRConv.forward`` a ``DGLGraph`` (``conv.py:49``) and DGL lazily builds
its in-edge CSC on the first ``update_all`` (``conv.py:63``) and caches it on the graph.  Here
the same happens explicitly: :func:`get_plan` builds (once per graph and device) the two row
CSRs of the layer — by destination for the forward / dQ pass and by source for the dK pass —
plus the chunked work items, and caches them on the graph object.

Accepted graphs:
  * :class:`Graph` — this package's lightweight COO graph (what the bench/tests use; DGL is not
    installed on the MI355X box);
  * a real ``DGLGraph`` (duck-typed: ``adj_tensors('csc')``, ``in_degrees``, ``out_degrees``,
    ``num_nodes``), when DGL is importable;
  * any object with ``edges() -> (src, dst)`` and ``num_nodes()``.

CSR order is DGL's: rows sorted stably, so edges inside a row keep ascending edge id (the
order DGL's CPU SpMM and torch's ``index_add`` accumulate in) — bit-exact indexing.
"""
import contextlib
import weakref
from dataclasses import dataclass
from typing import Optional

import torch

DEFAULT_CHUNK = 256     # max edges per work item (power-law rows are split above this)


class Graph:
    """Minimal homogeneous graph with the ``DGLGraph`` surface ``SIRConv`` needs
    (``conv.py:50-63``: ``local_scope``, ``in_degrees``, ``out_degrees``, ``num_nodes``, ``device``)."""

    def __init__(self, src, dst, num_nodes=None, batch_num_nodes=None):
        src = torch.as_tensor(src, dtype=torch.int64)
        dst = torch.as_tensor(dst, dtype=torch.int64)
        if src.shape != dst.shape or src.dim() != 1:
            raise ValueError("src and dst must be 1-D and of equal length")
        if num_nodes is None:
            num_nodes = int(max(src.max().item(), dst.max().item()) + 1) if src.numel() else 0
        self._src, self._dst, self._n = src, dst.to(src.device), int(num_nodes)
        if batch_num_nodes is None:
            batch_num_nodes = [self._n]
        self._bnn = torch.as_tensor(batch_num_nodes, dtype=torch.int64)
        if int(self._bnn.sum()) != self._n:
            raise ValueError("batch_num_nodes must sum to num_nodes")
        self.ndata, self.edata = {}, {}
        self._plans = {}

    # DGLGraph-compatible surface -----------------------------------------------------------
    def num_nodes(self):
        return self._n

    def num_edges(self):
        return int(self._src.numel())

    number_of_nodes = num_nodes
    number_of_edges = num_edges

    @property
    def device(self):
        return self._src.device

    def edges(self):
        return self._src, self._dst

    def in_degrees(self):
        return torch.bincount(self._dst, minlength=self._n)

    def out_degrees(self):
        return torch.bincount(self._src, minlength=self._n)

    def to(self, device):
        return Graph(self._src.to(device), self._dst.to(device), self._n, self._bnn)

    # batched graphs (dgl.batch semantics; used by GraphNorm, models/norm.py:16-17)
    def batch_num_nodes(self):
        return self._bnn

    @property
    def batch_size(self):
        return int(self._bnn.numel())

    @contextlib.contextmanager
    def local_scope(self):
        nd, ed = dict(self.ndata), dict(self.edata)
        try:
            yield
        finally:
            self.ndata, self.edata = nd, ed

    def __repr__(self):
        return f"Graph(num_nodes={self._n}, num_edges={self.num_edges()}, device={self.device})"


def batch(graphs):
    """``dgl.batch``: one graph whose node / edge ids are the inputs' concatenated with offsets."""
    offs, src, dst, bnn = 0, [], [], []
    for g in graphs:
        s_, d_ = g.edges()
        src.append(torch.as_tensor(s_, dtype=torch.int64) + offs)
        dst.append(torch.as_tensor(d_, dtype=torch.int64) + offs)
        n = int(g.num_nodes())
        bnn.append(n)
        offs += n
    if not graphs:
        return Graph(torch.zeros(0, dtype=torch.int64), torch.zeros(0, dtype=torch.int64), 0, [])
    return Graph(torch.cat(src), torch.cat(dst), offs, bnn)


def node_offsets(graph, device):
    """int64 [B+1] node offsets of a batched graph (cached per device)."""
    cache = getattr(graph, "_plans", None)
    key = ("offsets", str(device))
    if cache is not None and key in cache:
        return cache[key]
    bnn = torch.as_tensor(graph.batch_num_nodes(), dtype=torch.int64).to(device)
    off = torch.zeros(bnn.numel() + 1, dtype=torch.int64, device=device)
    torch.cumsum(bnn, 0, out=off[1:])
    if cache is not None:
        cache[key] = off
    return off


@dataclass
class RowCSR:
    """Row CSR + chunked work plan (layout documented in include/sirconv.h)."""
    n_rows: int
    rowptr: torch.Tensor          # int32 [n_rows+1]
    col: torch.Tensor             # int32 [E]   (node at the other end)
    eid: torch.Tensor             # int64 [E]   (edge ids, ascending inside a row)
    items: torch.Tensor           # int32 [n_items, 4] {row, e_begin, e_end, slot}
    splits: Optional[torch.Tensor]  # int32 [n_splits, 4] {row, slot_begin, n_slots, degree}
    n_items: int
    n_splits: int
    n_slots: int
    max_degree: int
    perm: Optional[torch.Tensor] = None   # int32 [E]: this CSR's position -> dst-CSR position


def build_row_csr(rows, cols, n_rows, chunk=DEFAULT_CHUNK):
    """Stable sort by ``rows`` (counting-sort semantics of DGL's COO->CSR), then the plan."""
    rows = rows.to(torch.int64)
    E = rows.numel()
    if E >= 2 ** 31 - 1:
        raise ValueError("int32 edge indices: E must be < 2^31")
    dev = rows.device
    if E:
        _, eid = torch.sort(rows, stable=True)
    else:
        eid = torch.zeros(0, dtype=torch.int64, device=dev)
    col = cols.to(torch.int64)[eid].to(torch.int32)
    deg = torch.bincount(rows, minlength=n_rows) if E else torch.zeros(n_rows, dtype=torch.int64, device=dev)
    rowptr = torch.zeros(n_rows + 1, dtype=torch.int64, device=dev)
    torch.cumsum(deg, 0, out=rowptr[1:])
    return plan_from_rowptr(rowptr, col, eid, n_rows, chunk)


def plan_from_rowptr(rowptr, col, eid, n_rows, chunk=DEFAULT_CHUNK):
    dev = rowptr.device
    rowptr = rowptr.to(torch.int64)
    deg = rowptr[1:] - rowptr[:-1]
    nch = torch.clamp((deg + chunk - 1) // chunk, min=1)
    n_items = int(nch.sum().item()) if n_rows else 0
    row_of = torch.repeat_interleave(torch.arange(n_rows, device=dev), nch)
    first = torch.cumsum(nch, 0) - nch
    k = torch.arange(n_items, device=dev) - first[row_of]
    eb = rowptr[row_of] + k * chunk
    ee = torch.minimum(eb + chunk, rowptr[row_of + 1])
    split_row = nch > 1
    split_item = split_row[row_of]
    slot = torch.full((n_items,), -1, dtype=torch.int64, device=dev)
    n_slots = int(split_item.sum().item()) if n_items else 0
    if n_slots:
        slot[split_item] = torch.arange(n_slots, device=dev)
    items = torch.stack([row_of, eb, ee, slot], 1).to(torch.int32).contiguous()
    srows = torch.nonzero(split_row).flatten()
    n_splits = int(srows.numel())
    splits = None
    if n_splits:
        s_n = nch[srows]
        s_begin = torch.cumsum(s_n, 0) - s_n
        splits = torch.stack([srows, s_begin, s_n, deg[srows]], 1).to(torch.int32).contiguous()
    return RowCSR(n_rows=n_rows, rowptr=rowptr.to(torch.int32).contiguous(), col=col.contiguous(),
                  eid=eid, items=items, splits=splits, n_items=n_items, n_splits=n_splits,
                  n_slots=n_slots, max_degree=int(deg.max().item()) if n_rows else 0)


def build_plans_native(src, dst, n_dst_rows, n_src_rows, chunk=DEFAULT_CHUNK):
    """Both row CSRs + plans + the src->dst position map on the device (``sir_csr_build``,
    ``sir_csr_perm``) with ONE host synchronisation (the plan sizes).  Same result as
    :func:`build_row_csr` bit for bit (stable order, same items/splits)."""
    from . import _native
    E = src.numel()
    if E >= 2 ** 31 - 1:
        raise ValueError("int32 edge indices: E must be < 2^31")
    d = _native.csr_build(dst, src, n_dst_rows, n_src_rows, chunk)
    s = _native.csr_build(src, dst, n_src_rows, n_dst_rows, chunk)
    perm = _native.csr_perm(d[2], s[2])
    counts = torch.stack([d[5], s[5]]).cpu().tolist()
    if counts[0][4] or counts[1][4]:
        raise ValueError(f"edge endpoint out of range: {counts[0][4]} bad edges "
                         f"(dst must be in [0, {n_dst_rows}), src in [0, {n_src_rows}))")
    csrs = []
    for (rowptr, col, eid, items, splits, _), cnt, n in ((d, counts[0], n_dst_rows), (s, counts[1], n_src_rows)):
        n_items, n_splits, n_slots, max_deg = cnt[:4]
        csrs.append(RowCSR(n_rows=n, rowptr=rowptr, col=col, eid=eid, items=items[:n_items],
                           splits=splits[:n_splits] if n_splits else None, n_items=n_items,
                           n_splits=n_splits, n_slots=n_slots, max_degree=max_deg))
    csrs[1].perm = perm
    return csrs[0], csrs[1]


class GraphPlan:
    """Everything per (graph, device) that the SIRConv kernels need; built once and cached.

    On a GPU the plan is built by the native device builder (:func:`build_plans_native`); host
    plans (CPU tests) use the torch restatement (:func:`build_row_csr`)."""

    def __init__(self, src, dst, num_nodes, device, chunk=DEFAULT_CHUNK, csc=None):
        self.num_nodes = int(num_nodes)
        self.device = torch.device(device)
        src = src.to(self.device, torch.int64)
        dst = dst.to(self.device, torch.int64)
        self.num_edges = int(src.numel())
        if self.device.type == "cuda" and csc is None:
            self.dst, self.src = build_plans_native(src, dst, self.num_nodes, self.num_nodes, chunk)
        else:
            if self.num_edges:
                lo = int(torch.minimum(src.min(), dst.min()).item())
                hi = int(torch.maximum(src.max(), dst.max()).item())
                if lo < 0 or hi >= self.num_nodes:      # the kernels index node rows by these ids
                    raise ValueError(f"edge endpoint out of range [0, {self.num_nodes}): min {lo}, max {hi}")
            if csc is not None:             # a DGL-provided in-edge CSC (indptr, indices, eids)
                indptr, indices, eids = (t.to(self.device) for t in csc)
                self.dst = plan_from_rowptr(indptr, indices.to(torch.int32), eids.to(torch.int64),
                                            self.num_nodes, chunk)
            else:
                self.dst = build_row_csr(dst, src, self.num_nodes, chunk)
            self.src = build_row_csr(src, dst, self.num_nodes, chunk)
            # sign-mask backward: the mask is written in dst-CSR order; the src pass finds an
            # edge's mask through its dst-CSR position
            pos_in_dst = torch.empty(self.num_edges, dtype=torch.int64, device=self.device)
            pos_in_dst[self.dst.eid] = torch.arange(self.num_edges, device=self.device)
            self.src.perm = pos_in_dst[self.src.eid].to(torch.int32).contiguous()
        self.in_deg = (self.dst.rowptr[1:] - self.dst.rowptr[:-1]).to(torch.int64)
        self.out_deg = (self.src.rowptr[1:] - self.src.rowptr[:-1]).to(torch.int64)
        self._norms = {}

    def norms(self, agg):
        """``conv.py:51-57``: fp32 deg^-1/2 for ``sym`` (clamp(min=1)), else None (== ones)."""
        if agg != "sym":
            return None, None
        if "sym" not in self._norms:
            if self.device.type == "cuda":     # native: IEEE 1/sqrt == CPU torch.pow(d, -0.5) bits
                from . import _native
                in_norm = torch.empty(self.num_nodes, dtype=torch.float32, device=self.device)
                out_norm = torch.empty_like(in_norm)
                _native.degree_norms(self.dst.rowptr, self.src.rowptr, in_norm, out_norm)
            else:                              # host-side plans (tests) use the reference formula
                in_norm = torch.pow(self.in_deg.float().clamp(min=1), -0.5).contiguous()
                out_norm = torch.pow(self.out_deg.float().clamp(min=1), -0.5).contiguous()
            self._norms["sym"] = (in_norm, out_norm)
        return self._norms["sym"]

    def in_degree_f(self):
        """fp32 [V, 1] in-degree clamped at 1 (the mean's divisor, ``fn.mean``), cached with the norms."""
        if "deg" not in self._norms:
            rp = self.dst.rowptr
            self._norms["deg"] = (rp[1:] - rp[:-1]).clamp(min=1).to(torch.float32)[:, None]
        return self._norms["deg"]


_weak_plans = weakref.WeakKeyDictionary()


def get_plan(graph, device, chunk=DEFAULT_CHUNK):
    """Return the cached :class:`GraphPlan` of ``graph`` on ``device`` (build on first use)."""
    device = torch.device(device)
    key = (str(device), chunk)
    cache = getattr(graph, "_plans", None)
    if cache is None:
        try:
            cache = _weak_plans.setdefault(graph, {})
        except TypeError:
            cache = {}
    plan = cache.get(key)
    if plan is not None:
        return plan
    n = int(graph.num_nodes())
    csc = None
    if hasattr(graph, "adj_tensors"):          # DGLGraph
        csc = graph.adj_tensors("csc")
    src, dst = graph.edges()
    plan = GraphPlan(torch.as_tensor(src), torch.as_tensor(dst), n, device, chunk, csc=csc)
    cache[key] = plan
    return plan

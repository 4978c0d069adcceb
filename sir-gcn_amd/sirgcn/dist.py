"""Multi-GPU SIRConv: destination-range edge-cut over one node.

The reference is single-GPU (``*/train.py --gpu``); this is the MI355X-native scale-out of
the same layer (``conv.py:49-67``), one process per GPU over RCCL (``torch.distributed``
backend ``nccl``):

* **Partition.** Destination rows [0, V) are cut into ``world`` contiguous ranges holding
  ≈E/world in-edges each (prefix sum of in-degree).  Rank p owns rows [r_p, r_{p+1}): their
  features X, Q, S, Y, the in-edges into them (so S needs no reduction) and dX.
* **Forward exchange.** Messages need K[u] for any source u, so each rank projects its own
  rows' K and one **all-gather** builds K for every node.  Slabs are padded to the largest
  range (``max_rows``); source ids are remapped once, at plan time, to padded positions
  ``owner(u) * max_rows + (u - r_owner)`` so the kernels index the gathered buffer directly.
* **Backward exchange.** The dQ pass is local.  The dK pass runs over the rank's local edges
  grouped by source (all padded source rows) and yields partial dK for every node; one
  **reduce-scatter** (sum) returns each rank its own rows.  Weight gradients are summed with
  one **all-reduce** of a flat buffer (``allreduce_grads``).
* ``sym`` needs GLOBAL out-degrees: local out-degree histograms are **all-reduced** once per
  plan.

The per-rank edge work uses the same kernels/ABI as one GPU (``_native``).  A different
``backend`` object with the same three functions can be injected (the CPU gloo tests do).
"""
import torch
import torch.distributed as dist

from . import _native
from .graph import DEFAULT_CHUNK, build_row_csr


def _host_staged(group, t):
    """gloo cannot run these collectives on device tensors: stage through host memory
    (rehearsals / CPU tests only; RCCL runs them in place)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_gather_into(out, inp, group=None):
    if _host_staged(group, inp):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def reduce_scatter_into(out, inp, group=None):
    if _host_staged(group, inp):
        o = out.cpu()
        dist.reduce_scatter_tensor(o, inp.cpu(), op=dist.ReduceOp.SUM, group=group)
        out.copy_(o)
    else:
        dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)


def all_reduce_sum(t, group=None):
    if _host_staged(group, t):
        c = t.cpu()
        dist.all_reduce(c, group=group)
        t.copy_(c)
    else:
        dist.all_reduce(t, group=group)


def partition_rows(in_deg, world):
    """Row boundaries [0, r_1, ..., V] with ≈E/world in-edges per range (edge-balanced)."""
    V = in_deg.numel()
    E = int(in_deg.sum().item())
    cum = torch.cumsum(in_deg.to(torch.int64), 0)
    bounds = [0]
    for p in range(1, world):
        target = (E * p + world - 1) // world
        b = int(torch.searchsorted(cum, torch.tensor(target, dtype=torch.int64)).item()) + 1
        bounds.append(min(max(b, bounds[-1]), V))
    bounds.append(V)
    return bounds


class DistGraph:
    """One rank's share of a dst-range edge-cut, plus its kernel plans.

    Attributes used by the kernels: ``dst`` (RowCSR over local rows, col = padded src ids),
    ``src`` (RowCSR over all padded source rows, col = local dst rows, ``perm`` into ``dst``),
    ``norms(agg)``."""

    def __init__(self, src, dst, num_nodes, bounds, rank, world, device, chunk=DEFAULT_CHUNK,
                 group=None):
        self.num_nodes, self.rank, self.world = int(num_nodes), rank, world
        self.device = torch.device(device)
        self.bounds = list(bounds)
        self.row_begin, self.row_end = bounds[rank], bounds[rank + 1]
        self.n_rows = self.row_end - self.row_begin
        self.max_rows = max(bounds[p + 1] - bounds[p] for p in range(world))
        self.padded_rows = self.max_rows * world
        self.group = group
        src = torch.as_tensor(src, dtype=torch.int64).to(self.device)
        dst = torch.as_tensor(dst, dtype=torch.int64).to(self.device)
        sel = (dst >= self.row_begin) & (dst < self.row_end)
        lsrc, ldst = src[sel], dst[sel] - self.row_begin          # edge-id order preserved
        self.num_local_edges = int(lsrc.numel())
        bt = torch.tensor(self.bounds, dtype=torch.int64, device=self.device)
        owner = torch.searchsorted(bt, lsrc, right=True) - 1
        psrc = owner * self.max_rows + (lsrc - bt[owner])          # padded source position
        self.dst = build_row_csr(ldst, psrc, self.n_rows, chunk)
        self.src = build_row_csr(psrc, ldst, self.padded_rows, chunk)
        E = self.num_local_edges
        pos_in_dst = torch.empty(E, dtype=torch.int64, device=self.device)
        pos_in_dst[self.dst.eid] = torch.arange(E, device=self.device)
        self.src.perm = pos_in_dst[self.src.eid].to(torch.int32).contiguous()
        self.in_deg = (self.dst.rowptr[1:] - self.dst.rowptr[:-1]).to(torch.int64)
        # global out-degree in padded layout: local histograms summed over ranks
        out_local = (self.src.rowptr[1:] - self.src.rowptr[:-1]).to(torch.int64)
        if world > 1:
            all_reduce_sum(out_local, group=group)
        self.out_deg = out_local
        self._norms = {}

    @classmethod
    def from_global(cls, src, dst, num_nodes, rank, world, device, chunk=DEFAULT_CHUNK, group=None):
        in_deg = torch.bincount(torch.as_tensor(dst, dtype=torch.int64), minlength=num_nodes)
        return cls(src, dst, num_nodes, partition_rows(in_deg, world), rank, world, device, chunk, group)

    def norms(self, agg):
        """``conv.py:51-57`` with global degrees: (in_norm of local rows, out_norm of padded rows)."""
        if agg != "sym":
            return None, None
        if "sym" not in self._norms:
            in_norm = torch.pow(self.in_deg.float().clamp(min=1), -0.5).contiguous()
            out_norm = torch.pow(self.out_deg.float().clamp(min=1), -0.5).contiguous()
            if self.device.type == "cuda":   # same bits as the CPU reference (sir_degree_norms)
                in_norm = torch.empty(self.n_rows, dtype=torch.float32, device=self.device)
                out_norm = torch.empty(self.padded_rows, dtype=torch.float32, device=self.device)
                _native.degree_norms(self.dst.rowptr, None, in_norm, None)
                rp = torch.zeros(self.padded_rows + 1, dtype=torch.int64, device=self.device)
                torch.cumsum(self.out_deg, 0, out=rp[1:])
                _native.degree_norms(rp.to(torch.int32), None, out_norm, None)
            self._norms["sym"] = (in_norm, out_norm)
        return self._norms["sym"]


class DistEdgeAggregate(torch.autograd.Function):
    """S_local = update_all(...) over the local in-edges; K all-gathered inside, dK
    reduce-scattered inside the backward."""

    @staticmethod
    def forward(ctx, Q, K_local, plan, H, agg, act, slope, backend, use_mask):
        dev = Q.device
        K_send = torch.zeros((plan.max_rows, H), device=dev, dtype=torch.float32)
        K_send[:plan.n_rows] = K_local
        K_all = torch.empty((plan.padded_rows, H), device=dev, dtype=torch.float32)
        if plan.world > 1:
            all_gather_into(K_all, K_send, group=plan.group)
        else:
            K_all.copy_(K_send)
        in_norm, out_norm = plan.norms(agg)
        S = torch.empty((plan.n_rows, H), device=dev, dtype=torch.float32)
        n_slots = max(plan.dst.n_slots, plan.src.n_slots)
        partial = torch.empty((max(n_slots, 1) * H,), device=dev, dtype=torch.float32) if n_slots else None
        nw = _native.mask_words(H, act) if (use_mask and backend is _native) else 0
        mask = None
        if nw and (Q.requires_grad or K_local.requires_grad):
            mask = torch.empty((max(plan.dst.col.numel(), 1) * nw,), device=dev, dtype=torch.int64)
        Qc = Q.contiguous().float()
        backend.edge_agg_fwd(plan.dst, Qc, K_all, in_norm, out_norm, agg, act, slope, S, partial, mask)
        if mask is not None:
            ctx.save_for_backward(mask)
        else:
            ctx.save_for_backward(Qc, K_all)
        ctx.masked = mask is not None
        ctx.plan, ctx.H, ctx.agg, ctx.act, ctx.slope, ctx.backend = plan, H, agg, act, slope, backend
        return S

    @staticmethod
    def backward(ctx, dS):
        plan, H, agg, act, slope, backend = ctx.plan, ctx.H, ctx.agg, ctx.act, ctx.slope, ctx.backend
        dev = dS.device
        G = dS.contiguous().float()
        if ctx.masked:
            (mask,) = ctx.saved_tensors
            Q = K_all = None
        else:
            Q, K_all = ctx.saved_tensors
            mask = None
        in_norm, out_norm = plan.norms(agg)
        n_slots = max(plan.dst.n_slots, plan.src.n_slots)
        partial = torch.empty((max(n_slots, 1) * H,), device=dev, dtype=torch.float32) if n_slots else None
        dQ = torch.empty((plan.n_rows, H), device=dev, dtype=torch.float32)
        Gm = torch.empty((plan.n_rows, H), device=dev, dtype=torch.float32) if agg == "mean" else None
        backend.edge_agg_bwd_dst(plan.dst, Q, K_all, G, in_norm, out_norm, agg, act, slope, dQ, Gm, partial, mask)
        dK_all = torch.empty((plan.padded_rows, H), device=dev, dtype=torch.float32)
        backend.edge_agg_bwd_src(plan.src, K_all, Q, Gm if Gm is not None else G, out_norm, in_norm,
                                 agg, act, slope, dK_all, partial, mask)
        dK_mine = torch.empty((plan.max_rows, H), device=dev, dtype=torch.float32)
        if plan.world > 1:
            reduce_scatter_into(dK_mine, dK_all, group=plan.group)
        else:
            dK_mine.copy_(dK_all)
        return dQ, dK_mine[:plan.n_rows], None, None, None, None, None, None, None


class DistSIRConv(torch.nn.Module):
    """Wraps a :class:`sirgcn.SIRConv` (same parameters / state_dict) for the edge-cut layout.

    ``forward(dgraph, feat_local)`` takes this rank's rows of X and returns its rows of Y.
    Call :meth:`allreduce_grads` after ``backward`` (data-parallel weight gradients)."""

    def __init__(self, conv, backend=None, use_mask=True):
        super().__init__()
        self.conv = conv
        self.backend = backend if backend is not None else _native
        self.use_mask = use_mask

    def forward(self, dgraph, feat):
        from .conv import activation_code
        c = self.conv
        if c._agg_type not in ("sum", "mean", "sym"):
            raise NotImplementedError(f"DistSIRConv: agg_type={c._agg_type!r}")
        if feat.shape[0] != dgraph.n_rows:
            raise ValueError(f"feat has {feat.shape[0]} rows, rank owns {dgraph.n_rows}")
        act, slope = activation_code(c.activation)
        H = c.linear_query.out_features
        Q = c.dropout(c.linear_query(feat))
        K = c.dropout(c.linear_key(feat))
        S = DistEdgeAggregate.apply(Q, K, dgraph, H, c._agg_type, act, slope, self.backend, self.use_mask)
        return c.linear_relation(S)

    def allreduce_grads(self, group=None):
        params = [p for p in self.conv.parameters() if p.grad is not None]
        if not params or not dist.is_initialized() or dist.get_world_size(group) == 1:
            return
        flat = torch.cat([p.grad.reshape(-1) for p in params])
        all_reduce_sum(flat, group=group)
        off = 0
        for p in params:
            n = p.grad.numel()
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
            off += n

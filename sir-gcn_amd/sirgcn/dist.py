"""Multi-GPU SIRConv: destination-range edge-cut over one node.

The reference is single-GPU (``*/train.py --gpu``); this is the MI355X-native scale-out of
the same layer (``conv.py:49-67``), one process per GPU over RCCL (``torch.distributed``
backend ``nccl``):

* **Partition.** Destination rows [0, V) are cut into ``world`` contiguous ranges holding
  ≈E/world in-edges each (prefix sum of in-degree).  Rank p owns rows [r_p, r_{p+1}): their
  features X, Q, S, Y, the in-edges into them (so S needs no reduction) and dX.
* **Halo layout.** A message u→v needs K[u].  Rank p's *halo* is the set of remote sources of its
  in-edges.  Every owner's row range is cut into ``chunks`` parts (``part_bounds``), and a halo row
  belongs to chunk c when it lies in part c of its owner's range; the halo is stored CHUNK-MAJOR:
  ``K_ext = [own rows | chunk 0 | chunk 1 | ...]``, each chunk holding its part of every owner's
  block in owner order.  Edge columns are remapped once, at plan time, to positions in ``K_ext``,
  so the single-GPU kernels run on it unchanged.
* **Forward: a pipelined exchange.**  K is projected part by part of the own range, and chunk c
  (the rows of part c that peers need) is packed and sent as soon as part c exists — ``chunks``
  sparse all-to-alls (RCCL alltoallv over the xGMI mesh: every chunk moves rows to EVERY peer, so
  each one uses all links at once).  The edges of each destination row are stored in segments by
  source — own sources and halo chunk 0 first, then the edges whose halo row is in chunk 1, 2, ...
  — and the edge pass runs segment by segment as the chunks land (``SIR_AGG_ACCUMULATE``: S[v] +=
  the segment's sum); the Q GEMM runs under the first chunk.  Every row sums its segments in the
  same fixed order, so the result is deterministic (not bit-identical to one GPU, whose rows sum in
  edge id order: tests hold it to the parity bar).  On the power-law S2 graph the halo is 1.15 M
  rows per rank at 8 ranks against the 1.77 M a dense all-gather moves.
* **Backward: the transpose, also pipelined.**  The dK pass runs first over the HALO rows of
  ``K_ext``, chunk by chunk, each chunk's partial dK sent back to its owners (reverse alltoallv) as
  soon as it is computed; the dQ pass and the dK pass over the own rows (one launch, as on one GPU)
  and the dW_R / dW_Q GEMMs run under the exchange.  Reverse chunk c carries only rows of the
  owner's part c, so part c's dK is completed (one gather-based segment sum over [own partial |
  received rows], fixed order, no atomics) as soon as chunk c lands, and its dX rows follow at once
  as ONE K = 2H GEMM on [dQ | dK] against [W_Q; W_K] (with dW_K's partial over the part).
* **Weight gradients**: reduced inside the backward with ``reduce_in_backward=True`` — dW_R / db_R
  and dW_Q / db_Q start their all-reduce under the exchange, dW_K after the last part — else one
  all-reduce of a flat buffer (``allreduce_grads``).
* **Feature dropout** (``conv.py:35,60-61``, training with p > 0): Q and K draw hashed masks from
  two device seeds in the GEMM epilogues, hashed with the GLOBAL row index (independent masks per
  rank).  The backward edge passes run without it and the owner applies the masks to its own dQ /
  dK rows once complete (``sir_dropout_apply``): a halo row's dK partial is summed over ranks
  before the mask of its owner can apply.
* **agg_type='max'** (``conv.py:46-47``): the halo K rows are gathered by the same chunked
  exchange (``HaloGather``, its backward the reverse exchange) and the fused max layer
  (``edgemlp.EdgeMaxLinearQK``) runs on [own | halo] rows.  Its Q / K dropout is the same hashed
  mask (``HashedDropout``, seeds mixed with the rank's first global row), applied to the own rows
  before the gather, so ranks seeded alike still draw independent masks.
* **Autocast** (``DistSIRConvFunction16``): 16-bit K_ext rows, edge passes and both exchanges in
  the 16-bit type — half the wire bytes.
* ``sym`` needs GLOBAL out-degrees: own-row out-degree histograms are completed by the same reverse
  exchange and forwarded to the halos (plan time, once).

The per-rank edge work uses the same kernels/ABI as one GPU (``_native``).  A different
``backend`` object with the same three edge functions can be injected (the CPU gloo tests do).
"""
import dataclasses

import torch
import torch.distributed as dist

from . import _native, linalg
from .conv import EdgeAggregate, _slots, _tn, _weight_and_bias_grad, _weight_and_bias_grad16, activation_code
from .graph import DEFAULT_CHUNK, build_plans_native, build_row_csr

DEFAULT_EXCHANGE_CHUNKS = 4


def _host_staged(group, t):
    """gloo cannot run these collectives on device tensors: stage through host memory
    (rehearsals / CPU tests only; RCCL runs them in place)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_to_all_rows(out, inp, out_splits, in_splits, group=None, async_op=False):
    """``out`` ← rows of every peer's ``inp`` (RCCL alltoallv).  Returns a waitable or None.
    ``group`` may also be an in-process communicator with the same method (tests)."""
    if hasattr(group, "all_to_all_rows"):
        return group.all_to_all_rows(out, inp, out_splits, in_splits, async_op=async_op)
    if _host_staged(group, inp):
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
        return None
    return dist.all_to_all_single(out, inp, out_splits, in_splits, group=group, async_op=async_op)


def all_reduce_sum(t, group=None):
    if _host_staged(group, t):
        c = t.cpu()
        dist.all_reduce(c, group=group)
        t.copy_(c)
    else:
        dist.all_reduce(t, group=group)


# per-row cost of the edge-cut layer in units of one in-edge: the node-row work (the five projection
# GEMMs ~4 ns, the halo packing, the segments' read-modify-writes of S and the dK completion ~4 ns per
# row at H = 256) against the edge passes' ~0.31 ns per edge (the S2 profile, tools/dist_model.py: the
# slowest of 8 ranks 3.53 ms at 12, 3.50 at 20-24, 3.51 at 32); an edge-only cut left the slowest rank
# of S2 at 8 ranks with 8 % more rows than the mean
ROW_WEIGHT = 24


def partition_rows(in_deg, world, row_weight=ROW_WEIGHT):
    """Row boundaries [0, r_1, ..., V] with ≈equal cost per range, cost = in-edges + row_weight per row
    (row_weight 0: edge-balanced)."""
    in_deg = in_deg.cpu()                  # plan time: a few host syncs, any device
    V = in_deg.numel()
    cum = torch.cumsum(in_deg.to(torch.int64) + int(row_weight), 0)
    E = int(cum[-1].item()) if V else 0
    bounds = [0]
    for p in range(1, world):
        target = (E * p + world - 1) // world
        b = int(torch.searchsorted(cum, torch.tensor(target, dtype=torch.int64)).item()) + 1
        bounds.append(min(max(b, bounds[-1]), V))
    bounds.append(V)
    return bounds


def _range_items(rows, begin, end, chunk):
    """Work items {row, e_begin, e_end, slot} over explicit edge ranges [begin, end) of ``rows``
    (ascending), ranges longer than ``chunk`` split into slotted items, and their splits {row,
    slot_begin, n_slots, degree} — ``graph.plan_from_rowptr`` for one segment of every row."""
    dev = rows.device
    deg = end - begin
    nch = torch.clamp((deg + chunk - 1) // chunk, min=1)
    n_items = int(nch.sum().item()) if rows.numel() else 0
    idx = torch.repeat_interleave(torch.arange(rows.numel(), device=dev), nch)
    first = torch.cumsum(nch, 0) - nch
    k = torch.arange(n_items, device=dev) - first[idx]
    eb = begin[idx] + k * chunk
    ee = torch.minimum(eb + chunk, end[idx])
    split_row = nch > 1
    split_item = split_row[idx]
    slot = torch.full((n_items,), -1, dtype=torch.int64, device=dev)
    n_slots = int(split_item.sum().item()) if n_items else 0
    if n_slots:
        slot[split_item] = torch.arange(n_slots, device=dev)
    items = torch.stack([rows[idx], eb, ee, slot], 1).to(torch.int32).contiguous()
    srow = torch.nonzero(split_row).flatten()
    splits = None
    if srow.numel():
        s_n = nch[srow]
        s_begin = torch.cumsum(s_n, 0) - s_n
        splits = torch.stack([rows[srow], s_begin, s_n, deg[srow]], 1).to(torch.int32).contiguous()
    return items, splits, n_items, int(srow.numel()), n_slots


def _row_slice(csr, r0, r1):
    """The work items (and split rows) of rows [r0, r1) of a plan: a view of ``csr`` (items and
    splits are sorted by row; slots keep their global numbering, so the full partial buffer serves)."""
    it = csr.items[:, 0].contiguous()
    bnd = torch.tensor([r0, r1], dtype=it.dtype, device=it.device)
    a, b = (int(x) for x in torch.searchsorted(it, bnd).tolist())
    sp, ns = None, 0
    if csr.n_splits:
        sr = csr.splits[:, 0].contiguous()
        c, d = (int(x) for x in torch.searchsorted(sr, bnd.to(sr.dtype)).tolist())
        if d > c:
            sp, ns = csr.splits[c:d], d - c
    return dataclasses.replace(csr, items=csr.items[a:b], n_items=b - a, splits=sp, n_splits=ns)


class DistGraph:
    """One rank's share of a dst-range edge-cut, its chunked halo exchange plan and kernel plans.

    ``src``/``dst`` may be the global edge list or any superset of this rank's in-edges; edges
    whose destination is outside [row_begin, row_end) are ignored.  Collective at construction
    (every rank of ``group`` must build its DistGraph together, with the same ``chunks``).

    Kernel-facing attributes: ``dst`` (RowCSR over own rows, col = K_ext positions; each row's
    edges in segment order), ``src`` (RowCSR over K_ext rows, col = own rows, ``perm`` into
    ``dst``), ``segments`` (the forward's per-segment views of ``dst``), ``src_halo`` / ``src_own``
    (the dK pass's per-chunk / own-row views of ``src``), ``norms(agg)``.
    Exchange plan, per chunk c: ``recv_splits[c]`` (halo rows per owner), ``send_splits[c]`` /
    ``send_idx[c]`` (own rows each peer reads, in the peer's halo order), ``halo_off[c]``."""

    def __init__(self, src, dst, num_nodes, bounds, rank, world, device, chunk=DEFAULT_CHUNK,
                 group=None, chunks=None):
        self.num_nodes, self.rank, self.world = int(num_nodes), rank, world
        self.device = torch.device(device)
        self.bounds = list(bounds)
        self.row_begin, self.row_end = bounds[rank], bounds[rank + 1]
        self.n_rows = n = self.row_end - self.row_begin
        self.group = group
        C = (DEFAULT_EXCHANGE_CHUNKS if chunks is None else int(chunks)) if world > 1 else 0
        self.chunks = C
        # own rows of exchange chunk c: [part_bounds[c], part_bounds[c + 1]) (local row x is in part (x C) // n)
        self.part_bounds = [-(-c * n // C) for c in range(C + 1)] if C else [0, n]
        dev = self.device
        src = torch.as_tensor(src, dtype=torch.int64).to(dev)
        dst = torch.as_tensor(dst, dtype=torch.int64).to(dev)
        sel = (dst >= self.row_begin) & (dst < self.row_end)
        lsrc, ldst = src[sel], dst[sel] - self.row_begin          # edge-id order preserved
        self.num_local_edges = E = int(lsrc.numel())
        local = (lsrc >= self.row_begin) & (lsrc < self.row_end)
        halo = torch.unique(lsrc[~local])                          # sorted -> grouped by owner
        self.n_halo = int(halo.numel())
        self.n_ext = n + self.n_halo
        bt = torch.tensor(self.bounds, dtype=torch.int64, device=dev)
        owner = torch.searchsorted(bt, halo, right=True) - 1
        # ---- chunk-major halo order: chunk c of owner q = the requested rows in the c-th of C equal
        # parts of q's row RANGE, so that an owner can send chunk c as soon as the K rows of its own
        # range part c are projected, and complete the dK of that part as soon as chunk c's reverse
        # exchange lands (the synthetic graphs relabel node ids at random: the parts hold similar
        # numbers of requested rows) ----
        if self.n_halo:
            lo_q = bt[owner]
            hchunk = ((halo - lo_q) * C) // (bt[owner + 1] - lo_q)
            key = hchunk * world + owner
            order = torch.argsort(key, stable=True)
            new_pos = torch.empty_like(order)
            new_pos[order] = torch.arange(self.n_halo, device=dev)
            rs = torch.bincount(key, minlength=C * world).view(C, world).cpu().tolist()
            self.halo_ids = halo[order]
        else:
            rs = [[0] * world for _ in range(C)]
            self.halo_ids = halo
        self.recv_splits = rs
        off = [0]
        for c in range(C):
            off.append(off[-1] + sum(rs[c]))
        self.halo_off = off
        # ---- who reads my rows: exchange the requests once, split them by the same rule ----
        self.send_splits = [[0] * world for _ in range(C)]
        self.send_idx = [torch.zeros(0, dtype=torch.int64, device=dev) for _ in range(C)]
        if world > 1:
            req_cnt = torch.bincount(owner, minlength=world)
            sc_t = torch.empty_like(req_cnt)
            all_to_all_rows(sc_t, req_cnt, [1] * world, [1] * world, group=group)
            sc = sc_t.cpu().tolist()
            req = torch.empty(sum(sc), dtype=torch.int64, device=dev)
            all_to_all_rows(req, halo.contiguous(), sc, req_cnt.cpu().tolist(), group=group)
            parts = [t - self.row_begin for t in torch.split(req, sc)]      # ascending local rows per peer
            qb = torch.tensor(self.part_bounds, dtype=torch.int64, device=dev)
            cuts = [torch.searchsorted(t, qb).cpu().tolist() for t in parts]
            for c in range(C):
                idx_c = []
                for q in range(world):
                    a, b = cuts[q][c], cuts[q][c + 1]                     # requests inside my part c
                    self.send_splits[c][q] = b - a
                    idx_c.append(parts[q][a:b])
                self.send_idx[c] = torch.cat(idx_c).contiguous()
            allidx = torch.cat(self.send_idx)
            if allidx.numel():
                lo, hi = int(allidx.min()), int(allidx.max())
                if lo < 0 or hi >= n:
                    raise RuntimeError(f"rank {rank}: peers requested rows outside [0, {n})")
        self._send_parts = [list(torch.split(self.send_idx[c], self.send_splits[c])) for c in range(C)]
        # the backward's received dK partials, one buffer after dK_ext: chunk c at recv_off[c]; the own
        # rows' complete dK is ONE segment sum over [own partial, chunk 0 peers 0.., chunk 1 ...] per row
        # (a gather: no atomics, fixed order) — recv_plan rows = own rows, col = row positions in
        # [dK_ext | received]
        roff = [0]
        for c in range(C):
            roff.append(roff[-1] + int(self.send_idx[c].numel()))
        self.recv_off = roff
        tgt = torch.cat([torch.arange(n, device=dev)] + [t for t in self.send_idx])
        pos = torch.cat([torch.arange(n, device=dev), self.n_ext + torch.arange(roff[-1], device=dev)])
        self.recv_plan = build_row_csr(tgt, pos, n, chunk)
        # ---- edge columns in K_ext, segments (0: own source AND halo chunk 0, which lands under the
        # Q GEMM and the packing of the later chunks; c >= 1: halo chunk c) ----
        if self.n_halo:
            hp = torch.searchsorted(halo, lsrc).clamp_(max=self.n_halo - 1)
            col = torch.where(local, lsrc - self.row_begin, n + new_pos[hp])
            seg = torch.where(local, torch.zeros_like(lsrc), hchunk[hp])
        else:
            col = lsrc - self.row_begin
            seg = torch.zeros_like(lsrc)
        NS = max(C, 1)
        so = torch.argsort(seg, stable=True)     # the row sort below keeps (segment, edge id) order inside a row
        col, ldst, seg = col[so], ldst[so], seg[so]
        # ---- kernel plans over the K_ext layout ----
        if dev.type == "cuda":
            self.dst, self.src = build_plans_native(col, ldst, n, self.n_ext, chunk)
        else:
            self.dst = build_row_csr(ldst, col, n, chunk)
            self.src = build_row_csr(col, ldst, self.n_ext, chunk)
            pos_in_dst = torch.empty(E, dtype=torch.int64, device=dev)
            pos_in_dst[self.dst.eid] = torch.arange(E, device=dev)
            self.src.perm = pos_in_dst[self.src.eid].to(torch.int32).contiguous()
        # forward segments: per (row, segment) edge ranges of the dst CSR
        cnt_rs = torch.bincount(ldst * NS + seg, minlength=n * NS)[:n * NS].view(n, NS)
        rp = self.dst.rowptr[:-1].to(torch.int64)
        ends = rp[:, None] + torch.cumsum(cnt_rs, 1)
        begins = ends - cnt_rs
        self.segments = []
        for s in range(NS):
            r = torch.arange(n, device=dev) if s == 0 else torch.nonzero(cnt_rs[:, s]).flatten()
            it, sp, ni, ns, nsl = _range_items(r, begins[r, s], ends[r, s], chunk)
            self.segments.append(dataclasses.replace(self.dst, items=it, n_items=ni, splits=sp, n_splits=ns,
                                                     n_slots=nsl))
        self.src_own = _row_slice(self.src, 0, n)
        self.src_halo = [_row_slice(self.src, n + off[c], n + off[c + 1]) for c in range(C)]
        self.in_deg = (self.dst.rowptr[1:] - self.dst.rowptr[:-1]).to(torch.int64)
        self.local_out_deg = (self.src.rowptr[1:] - self.src.rowptr[:-1]).to(torch.int64)
        self._out_deg = None
        self._norms = {}
        self._deg_f = None       # fp32 in-degree of own rows (MEAN)

    @classmethod
    def from_global(cls, src, dst, num_nodes, rank, world, device, chunk=DEFAULT_CHUNK, group=None, chunks=None):
        in_deg = torch.bincount(torch.as_tensor(dst, dtype=torch.int64), minlength=num_nodes)
        return cls(src, dst, num_nodes, partition_rows(in_deg, world), rank, world, device, chunk, group, chunks)

    # ---- exchanges (rows of [n, F] tensors), one chunk at a time ----
    def halo_rows(self, c):
        """K_ext row range of halo chunk c."""
        return self.n_rows + self.halo_off[c], self.n_rows + self.halo_off[c + 1]

    def gather_chunk(self, c, own, ext, async_op=False):
        """ext[halo chunk c] ← the owners' rows of ``own`` (forward alltoallv)."""
        a, b = self.halo_rows(c)
        send = own.index_select(0, self.send_idx[c])
        return all_to_all_rows(ext[a:b], send, self.recv_splits[c], self.send_splits[c], self.group, async_op)

    def scatter_chunk(self, c, ext, recv, async_op=False):
        """Reverse alltoallv of chunk c: recv (send_idx[c] order) ← the peers' halo rows of my nodes."""
        a, b = self.halo_rows(c)
        return all_to_all_rows(recv, ext[a:b].contiguous(), self.send_splits[c], self.recv_splits[c], self.group,
                               async_op)

    def add_received(self, c, own, recv):
        """own[send_idx[c][q]] += recv rows of peer q, peers in ascending order (deterministic: indices are
        unique within one peer's slice)."""
        for idx, part in zip(self._send_parts[c], torch.split(recv, self.send_splits[c])):
            if idx.numel():
                own.index_add_(0, idx, part)

    def own_range(self, c):
        """Own rows whose K rows exchange chunk c sends and whose dK it completes."""
        return self.part_bounds[c], self.part_bounds[c + 1]

    def recv_part(self, c):
        """``recv_plan`` restricted to the own rows of part c (their received rows all come with chunk c)."""
        if not hasattr(self, "_recv_parts"):
            self._recv_parts = [_row_slice(self.recv_plan, *self.own_range(k)) for k in range(self.chunks)]
        return self._recv_parts[c]

    def gather_halo(self, own, ext):
        """ext[n:] ← the owners' rows of ``own``, every chunk (synchronous)."""
        for c in range(self.chunks):
            self.gather_chunk(c, own, ext)

    def out_deg(self):
        """GLOBAL out-degree of every K_ext row (own + halo)."""
        if self._out_deg is None:
            deg = self.local_out_deg.clone()
            n = self.n_rows
            for c in range(self.chunks):
                recv = torch.empty(self.send_idx[c].numel(), dtype=torch.int64, device=self.device)
                self.scatter_chunk(c, deg, recv)
                self.add_received(c, deg[:n], recv)
            self.gather_halo(deg[:n], deg)
            self._out_deg = deg
        return self._out_deg

    def norms(self, agg):
        """``conv.py:51-57`` with global degrees: (in_norm of own rows, out_norm of K_ext rows)."""
        if agg != "sym":
            return None, None
        if "sym" not in self._norms:
            out_deg = self.out_deg()
            if self.device.type == "cuda":   # same bits as the CPU reference (sir_degree_norms)
                in_norm = torch.empty(self.n_rows, dtype=torch.float32, device=self.device)
                out_norm = torch.empty(self.n_ext, dtype=torch.float32, device=self.device)
                _native.degree_norms(self.dst.rowptr, None, in_norm, None)
                rp = torch.zeros(self.n_ext + 1, dtype=torch.int64, device=self.device)
                torch.cumsum(out_deg, 0, out=rp[1:])
                _native.degree_norms(rp.to(torch.int32), None, out_norm, None)
            else:
                in_norm = torch.pow(self.in_deg.float().clamp(min=1), -0.5).contiguous()
                out_norm = torch.pow(out_deg.float().clamp(min=1), -0.5).contiguous()
            self._norms["sym"] = (in_norm, out_norm)
        return self._norms["sym"]

    def deg_f(self):
        """fp32 max(in-degree, 1) of the own rows, [n, 1] (MEAN)."""
        if self._deg_f is None:
            self._deg_f = self.in_deg.clamp(min=1).to(torch.float32)[:, None]
        return self._deg_f

    def exchange_rows(self):
        """Rows this rank receives / sends per forward exchange (for reporting)."""
        return self.n_halo, int(sum(int(t.numel()) for t in self.send_idx))


def _workspace(plan, H, device):
    n = max(plan.dst.n_slots, plan.src.n_slots, *(s.n_slots for s in plan.segments))
    return torch.empty((max(n, 1) * H,), device=device, dtype=torch.float32) if n else None


def _segmented_forward(backend, dg, Q, K_ext, agg, act, slope, S, mask, works):
    """S = update_all(...) over the rank's in-edges, segment by segment as the halo chunks land:
    segment 0 (own sources and halo chunk 0) writes every row, segment c >= 1 adds its sum; each
    waits for its chunk (``works[c]``; None: already complete).  One segment per chunk, the own
    sources riding with chunk 0: chunk 0 lands while the Q GEMM and the packing of the later chunks
    run, and every extra segment costs a read-modify-write of S (tools/dist_model.py: -2 % per
    step at 8 ranks).  MEAN divides once, after the last segment."""
    in_norm, out_norm = dg.norms(agg)
    a = "sum" if agg == "mean" else agg
    partial = _workspace(dg, Q.shape[1], Q.device)
    for s, seg in enumerate(dg.segments):
        if s < len(works) and works[s] is not None:
            works[s].wait()
        backend.edge_agg_fwd(seg, Q, K_ext, in_norm, out_norm, a, act, slope, S, partial, mask, accumulate=s > 0)
    if agg == "mean":
        S.copy_(S / dg.deg_f())      # fp32 division, one rounding to S's dtype (DGL fn.mean)


def _chunked_backward(backend, dg, H, agg, act, slope, G, Q, K_ext, mask, dQ, dK_ext, recvs):
    """dK over the halo rows chunk by chunk, each chunk's rows sent back to their owners as soon as
    they are complete (returns the pending works), then dQ and the own rows' dK — in one launch in
    sign-mask mode on the native backend — under the exchange.  MEAN runs on G / deg (both passes
    read exactly those values, as the single-GPU layer does)."""
    in_norm, out_norm = dg.norms(agg)
    if agg == "mean":
        G = (G / dg.deg_f()).to(G.dtype)
        agg = "sum"
    partial = _workspace(dg, H, G.device)
    partial_s = _slots(dg.src, H, G.device)
    works = []
    for c in range(dg.chunks):
        backend.edge_agg_bwd_src(dg.src_halo[c], K_ext, Q, G, out_norm, in_norm, agg, act, slope, dK_ext,
                                 partial_s, mask)
        works.append(dg.scatter_chunk(c, dK_ext, recvs[c], async_op=True))
    if mask is not None and backend is _native and EdgeAggregate.dual:
        _native.edge_agg_bwd(dg.dst, dg.src_own, G, mask, in_norm, out_norm, agg, act, slope, dQ, dK_ext,
                             partial, partial_s)
    else:
        backend.edge_agg_bwd_dst(dg.dst, Q, K_ext, G, in_norm, out_norm, agg, act, slope, dQ, None, partial, mask)
        backend.edge_agg_bwd_src(dg.src_own, K_ext, Q, G, out_norm, in_norm, agg, act, slope, dK_ext, partial_s,
                                 mask)
    return works


def _backward_buffers(dg, H, dev, dtype):
    """dK_ext and the chunks' receive buffers as slices of ONE buffer [n_ext + received rows, H]."""
    big = torch.empty((dg.n_ext + dg.recv_off[-1], H), device=dev, dtype=dtype)
    recvs = [big[dg.n_ext + dg.recv_off[c]:dg.n_ext + dg.recv_off[c + 1]] for c in range(dg.chunks)]
    return big, big[:dg.n_ext], recvs


def _complete_dk_parts(dg, big, recvs, works, backend, out=None):
    """Yield (dK rows of own part c, a, b) as each reverse chunk lands: the rows of part c receive
    partials from chunk c only, summed in a fixed order (own partial, then peers ascending) — one
    native segment sum per part (a gather: no atomics), else per-peer index_add (unique indices per
    call: deterministic)."""
    n = dg.n_rows
    if not dg.chunks:
        if out is not None:
            out.copy_(big[:n])
            yield out, 0, n
        else:
            yield big[:n], 0, n
        return
    native = backend is _native and big.dtype == torch.float32
    if native:
        dK = out if out is not None else torch.empty((n, big.shape[1]), device=big.device, dtype=big.dtype)
        part = torch.empty((dg.recv_plan.n_slots * big.shape[1],), device=big.device) if dg.recv_plan.n_slots else None
    for c in range(dg.chunks):
        if works[c] is not None:
            works[c].wait()
        a, b = dg.own_range(c)
        if b <= a:
            continue
        if native:
            rp = dg.recv_part(c)
            _native.segment_sum(rp, big, dK, perm=rp.col, partial=part)
            yield dK[a:b], a, b
        else:
            own = big[:n]
            dg.add_received(c, own, recvs[c])
            if out is not None:
                out[a:b] = own[a:b]
                yield out[a:b], a, b
            else:
                yield own[a:b], a, b


def _complete_dk(dg, big, recvs, works, backend):
    """dK of the own rows = own partial + every peer's halo partial, in a fixed order (own, then chunk by
    chunk, peers ascending): one native segment sum gathering the rows of ``big`` (fp32), else per chunk
    and peer index_add (unique indices per call: deterministic)."""
    for c in range(dg.chunks):
        if works[c] is not None:
            works[c].wait()
    n = dg.n_rows
    if backend is _native and big.dtype == torch.float32 and dg.chunks:
        dK = torch.empty((n, big.shape[1]), device=big.device, dtype=big.dtype)
        rp = dg.recv_plan
        part = torch.empty((rp.n_slots * big.shape[1],), device=big.device) if rp.n_slots else None
        _native.segment_sum(rp, big, dK, perm=rp.col, partial=part)
        return dK
    dK = big[:n]
    for c in range(dg.chunks):
        dg.add_received(c, dK, recvs[c])
    return dK


_SEED_MIX = 0x2545F4914F6CDD1D        # odd 62-bit multiplier mixing a rank's global row offset into its seeds


def _drops(drop, row_begin=0):
    """(Q drop, K drop) of a (seeds, p) pair: two independent device seeds (or ints).  The kernels
    hash the LOCAL row index, so each rank's seeds are offset by a function of its first global row
    (``row_begin``): local row i of two ranks then draws independent bits, as the reference's
    nn.Dropout does over the whole [V, H] tensor (every rank draws the same seeds from its generator
    under the usual torch.manual_seed(same))."""
    if drop is None:
        return None, None
    seeds, p = drop
    off = (int(row_begin) * _SEED_MIX) % (1 << 62)
    if isinstance(seeds, torch.Tensor):
        if off:
            seeds = torch.bitwise_xor(seeds, off)
        return (seeds[0:1], p), (seeds[1:2], p)
    s0 = int(seeds) ^ off
    return (s0, p), ((s0 * 0x9E3779B97F4A7C15 + 1) % (1 << 62), p)


def _drop_at(drop, row0):
    """The K dropout of the own-row part starting at local row ``row0``: the K GEMM runs per part
    (its epilogue hashes the row index inside the part), so each part's seed is offset by ``row0``
    (part 0 keeps the rank's seed); the backward applies the same per-part masks to dK."""
    if drop is None or row0 == 0:
        return drop
    seed, p = drop
    off = (int(row0) * _SEED_MIX * 3) % (1 << 62)
    if isinstance(seed, torch.Tensor):
        return torch.bitwise_xor(seed, off), p
    return int(seed) ^ off, p


class _GradReducer:
    """Weight gradients all-reduced INSIDE the backward (``DistSIRConv(reduce_in_backward=True)``):
    dW_R / db_R and dW_Q / db_Q are queued on RCCL right after they are computed, under the reverse
    exchange; dW_K, the last one, at the end.  ``group=None`` with no process group: nothing."""

    def __init__(self, group):
        self.group = group
        self.pending = []

    def add(self, tensors):
        ts = [t for t in tensors if t is not None]
        if not ts:
            return
        if hasattr(self.group, "all_to_all_rows"):
            raise NotImplementedError("reduce_in_backward needs a torch.distributed process group")
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return                  # one process: its partial sums are the gradients (as allreduce_grads)
        flat = torch.cat([t.reshape(-1) for t in ts])
        if flat.is_cuda and not _host_staged(self.group, flat):
            work = dist.all_reduce(flat, group=self.group, async_op=True)     # RCCL, under the exchange
        else:
            all_reduce_sum(flat, group=self.group)                            # gloo rehearsals
            work = None
        self.pending.append((work, flat, ts))

    def finish(self):
        for work, flat, ts in self.pending:
            if work is not None:
                work.wait()
            off = 0
            for t in ts:
                k = t.numel()
                t.copy_(flat[off:off + k].view_as(t))
                off += k
        self.pending = []


class DistSIRConvFunction(torch.autograd.Function):
    """One rank's share of the whole layer, hand-scheduled around the two pipelined exchanges.

    forward : K_own = X W_K^T -> ``chunks`` halo alltoallvs queued ‖ Q = X W_Q^T + b_Q -> segment c
              (0: own sources + chunk 0) as chunk c lands -> Y = S W_R^T + b_R
    backward: G = dY W_R -> dK of halo chunk c -> its reverse alltoallv (each as soon as computed) ‖
              dQ pass + own-row dK, dW_R, db_R, dX = dQ W_Q, dW_Q, db_Q -> dK_own += received ->
              dX += dK W_K, dW_K.  Weight gradients are this rank's partial sums.
    ``drop``: (two device seeds, p) of the Q / K feature dropout (conv.py:60-61), or None."""

    @staticmethod
    def forward(ctx, X, W_Q, b_Q, W_K, W_R, b_R, dg, agg, act, slope, backend, use_mask, grad_on=True, drop=None,
                reduce=False):
        H = W_Q.shape[0]
        n = dg.n_rows
        ctx.reduce = reduce
        dev = X.device
        X = X.contiguous()
        dq, dk = _drops(drop, dg.row_begin)
        K_ext = torch.empty((dg.n_ext, H), device=dev, dtype=torch.float32)
        # K part by part: exchange chunk c carries only rows of part c, so it leaves as soon as they exist
        works = []
        for c in range(max(dg.chunks, 1)):
            a, b = dg.own_range(c)
            if b > a:
                linalg.mm_wt(X[a:b], W_K, out=K_ext[a:b], drop=_drop_at(dk, a))
            if c < dg.chunks:
                works.append(dg.gather_chunk(c, K_ext[:n], K_ext, async_op=True))
        Q = linalg.mm_wt(X, W_Q, b_Q, drop=dq)
        S = torch.empty((n, H), device=dev, dtype=torch.float32)
        training = grad_on and any(ctx.needs_input_grad[:6])     # grad mode passed in (see conv.py)
        nw = _native.mask_words(H, act) if (use_mask and training and backend is _native) else 0
        mask = torch.empty((max(dg.dst.col.numel(), 1) * nw,), device=dev, dtype=torch.int64) if nw else None
        _segmented_forward(backend, dg, Q, K_ext, agg, act, slope, S, mask, works)
        Y = linalg.mm_wt(S, W_R, b_R)
        if mask is not None:
            ctx.save_for_backward(X, W_Q, W_K, W_R, S, mask)
        else:
            ctx.save_for_backward(X, W_Q, W_K, W_R, S, Q, K_ext)
        ctx.masked = mask is not None
        ctx.dg, ctx.agg, ctx.act, ctx.slope, ctx.backend, ctx.drop = dg, agg, act, slope, backend, (dq, dk)
        ctx.has_bq, ctx.has_br = b_Q is not None, b_R is not None
        return Y

    @staticmethod
    def backward(ctx, dY):
        dg, agg, act, slope, backend = ctx.dg, ctx.agg, ctx.act, ctx.slope, ctx.backend
        dq, dk = ctx.drop
        if ctx.masked:
            X, W_Q, W_K, W_R, S, mask = ctx.saved_tensors
            Q = K_ext = None
        else:
            X, W_Q, W_K, W_R, S, Q, K_ext = ctx.saved_tensors
            mask = None
        H = W_R.shape[1]
        n = dg.n_rows
        dev = X.device
        dY = dY.contiguous()
        red = _GradReducer(dg.group) if ctx.reduce else None
        G = linalg.mm_w(dY, W_R)
        # dQ and the completed own-row dK side by side ([dQ | dK], as on one GPU): dX of each part is then
        # ONE K = 2H GEMM against [W_Q; W_K], written once (no dX read-modify-write per part)
        dQK = torch.empty((n, 2 * H), device=dev, dtype=torch.float32)
        dQ = dQK[:, :H]
        big, dK_ext, recvs = _backward_buffers(dg, H, dev, torch.float32)
        works = _chunked_backward(backend, dg, H, agg, act, slope, G, Q, K_ext, mask, dQ, dK_ext, recvs)
        if dq is not None:
            _native.dropout_apply(dQ, dq)
        dW_R, db_R = _weight_and_bias_grad(dY, S, ctx.needs_input_grad[4], ctx.has_br and ctx.needs_input_grad[5])
        if red is not None:
            red.add([dW_R, db_R])
        dW_Q, db_Q = _weight_and_bias_grad(dQ, X, ctx.needs_input_grad[1], ctx.has_bq and ctx.needs_input_grad[2])
        if red is not None:
            red.add([dW_Q, db_Q])
        dX = torch.empty((n, X.shape[1]), device=dev, dtype=torch.float32) if ctx.needs_input_grad[0] else None
        W_cat = torch.cat([W_Q, W_K], 0) if dX is not None else None
        # dK part by part as each reverse chunk lands: complete, mask, dX = [dQ | dK] [W_Q; W_K], dW_K += dK^T X
        dW_K = None
        for c, (dK, a, b) in enumerate(_complete_dk_parts(dg, big, recvs, works, backend, out=dQK[:, H:])):
            if dk is not None:
                _native.dropout_apply(dK, _drop_at(dk, a))
            if dX is not None:
                linalg.mm_w(dQK[a:b], W_cat, out=dX[a:b])
            if ctx.needs_input_grad[3]:
                part = _tn(dK, X[a:b])
                dW_K = part if dW_K is None else dW_K.add_(part)       # parts in order: deterministic
        if red is not None:
            red.add([dW_K])
            red.finish()
        return dX, dW_Q, db_Q, dW_K, dW_R, db_R, None, None, None, None, None, None, None, None, None


class DistSIRConvFunction16(torch.autograd.Function):
    """:class:`DistSIRConvFunction` under autocast (bf16 / fp16 ``dt``, the reference's AMP path):
    the single-GPU ``SIRConvFunction16`` dataflow per rank — 16-bit projections on the native
    16-bit MFMA GEMMs (X.to(dt) fused into the first one), 16-bit ``K_ext`` rows and edge passes
    (fp32 math inside) — with both pipelined halo exchanges in the 16-bit storage type: half the
    xGMI bytes of the fp32 layer.  Two roundings more than the single-GPU autocast layer, both within
    the AMP tolerance and pinned by ``tests/test_dist_gpu.py::test_autocast_edge_cut_16bit_wire``
    (default 4 chunks, sum / sym / mean): S is accumulated segment by segment in the 16-bit storage
    type (one rounding per halo chunk; ``mean`` divides the rounded sum), and the received dK rows
    are added in that type (one more rounding per peer)."""

    @staticmethod
    def forward(ctx, X, W_Q, b_Q, W_K, W_R, b_R, dg, agg, act, slope, backend, use_mask, grad_on, dt, drop=None,
                reduce=False):
        H = W_Q.shape[0]
        n = dg.n_rows
        ctx.reduce = reduce
        dev = X.device
        X = X.contiguous()
        dq, dk = _drops(drop, dg.row_begin)
        K_ext = torch.empty((dg.n_ext, H), device=dev, dtype=dt)
        Xh = X if X.dtype == dt else torch.empty(X.shape, dtype=dt, device=dev)
        works = []
        for c in range(max(dg.chunks, 1)):           # K part by part; chunk c leaves after part c
            a, b = dg.own_range(c)
            if b > a:
                if X.dtype == dt:
                    linalg.mm16_wt(X[a:b], W_K, None, dt, out=K_ext[a:b], drop=_drop_at(dk, a))
                else:       # X.to(dt) fused into the K GEMM's loads; the rounded X (for dW) written by it
                    linalg.mm16_wt(X[a:b], W_K, None, dt, acopy=Xh[a:b], out=K_ext[a:b], drop=_drop_at(dk, a))
            if c < dg.chunks:
                works.append(dg.gather_chunk(c, K_ext[:n], K_ext, async_op=True))
        Q = linalg.mm16_wt(Xh, W_Q, b_Q, dt, drop=dq)
        S = torch.empty((n, H), device=dev, dtype=dt)
        training = grad_on and any(ctx.needs_input_grad[:6])
        nw = _native.mask_words(H, act) if (use_mask and training and backend is _native) else 0
        mask = torch.empty((max(dg.dst.col.numel(), 1) * nw,), device=dev, dtype=torch.int64) if nw else None
        _segmented_forward(backend, dg, Q, K_ext, agg, act, slope, S, mask, works)
        Y = linalg.mm16_wt(S, W_R, b_R, dt)
        if mask is not None:
            ctx.save_for_backward(Xh, W_Q, W_K, W_R, S, mask)
        else:
            ctx.save_for_backward(Xh, W_Q, W_K, W_R, S, Q, K_ext)
        ctx.masked = mask is not None
        ctx.dg, ctx.agg, ctx.act, ctx.slope, ctx.backend, ctx.drop = dg, agg, act, slope, backend, (dq, dk)
        ctx.x_dtype, ctx.dt = X.dtype, dt
        ctx.has_bq, ctx.has_br = b_Q is not None, b_R is not None
        return Y

    @staticmethod
    def backward(ctx, dY):
        dg, agg, act, slope, backend, dt = ctx.dg, ctx.agg, ctx.act, ctx.slope, ctx.backend, ctx.dt
        dq, dk = ctx.drop
        if ctx.masked:
            Xh, W_Q, W_K, W_R, S, mask = ctx.saved_tensors
            Q = K_ext = None
        else:
            Xh, W_Q, W_K, W_R, S, Q, K_ext = ctx.saved_tensors
            mask = None
        H = W_R.shape[1]
        n = dg.n_rows
        dev = Xh.device
        dY = dY.contiguous().to(dt)
        red = _GradReducer(dg.group) if ctx.reduce else None
        G = linalg.mm16_w(dY, W_R, dt)
        dQ = torch.empty((n, H), device=dev, dtype=dt)
        big, dK_ext, recvs = _backward_buffers(dg, H, dev, dt)
        works = _chunked_backward(backend, dg, H, agg, act, slope, G, Q, K_ext, mask, dQ, dK_ext, recvs)
        if dq is not None:
            _native.dropout_apply(dQ, dq)
        dW_R = db_R = None
        if ctx.needs_input_grad[4] or ctx.needs_input_grad[5]:
            dW_R, db_R = _weight_and_bias_grad16(dY, S, ctx.needs_input_grad[4], ctx.has_br and ctx.needs_input_grad[5])
        if red is not None:
            red.add([dW_R, db_R])
        dX = linalg.mm16_w(dQ, W_Q, dt, out_dtype=torch.float32) if ctx.needs_input_grad[0] else None
        dW_Q = db_Q = None
        if ctx.needs_input_grad[1] or (ctx.has_bq and ctx.needs_input_grad[2]):
            dW_Q, db_Q = _weight_and_bias_grad16(dQ, Xh, True, ctx.has_bq and ctx.needs_input_grad[2])
        if red is not None:
            red.add([dW_Q, db_Q])
        dW_K = None
        for c, (dK, a, b) in enumerate(_complete_dk_parts(dg, big, recvs, works, backend)):
            if dk is not None:
                _native.dropout_apply(dK, _drop_at(dk, a))
            if dX is not None:
                dX[a:b] += linalg.mm16_w(dK, W_K, dt, out_dtype=torch.float32)
            if ctx.needs_input_grad[3]:
                part = _weight_and_bias_grad16(dK, Xh[a:b], True, False)[0]
                dW_K = part if dW_K is None else dW_K.add_(part)
        if dX is not None:
            dX = dX.to(ctx.x_dtype)
        if red is not None:
            red.add([dW_K])
            red.finish()
        return dX, dW_Q, db_Q, dW_K, dW_R, db_R, None, None, None, None, None, None, None, None, None, None


class DistEdgeAggregate(torch.autograd.Function):
    """Modular variant (layers the fused Functions do not take: other dtypes, tuple features): S_local
    = update_all(...) over the local in-edges from Q (own rows) and K (own rows), with the same
    pipelined exchanges inside."""

    @staticmethod
    def forward(ctx, Q, K_local, dg, H, agg, act, slope, backend, use_mask, grad_on=True):
        dev = Q.device
        n = dg.n_rows
        K_ext = torch.empty((dg.n_ext, H), device=dev, dtype=torch.float32)
        K_ext[:n] = K_local
        works = [dg.gather_chunk(c, K_ext[:n], K_ext, async_op=True) for c in range(dg.chunks)]
        S = torch.empty((n, H), device=dev, dtype=torch.float32)
        nw = _native.mask_words(H, act) if (use_mask and backend is _native) else 0
        mask = None
        if nw and grad_on and (Q.requires_grad or K_local.requires_grad):
            mask = torch.empty((max(dg.dst.col.numel(), 1) * nw,), device=dev, dtype=torch.int64)
        Qc = Q.contiguous().float()
        _segmented_forward(backend, dg, Qc, K_ext, agg, act, slope, S, mask, works)
        if mask is not None:
            ctx.save_for_backward(mask)
        else:
            ctx.save_for_backward(Qc, K_ext)
        ctx.masked = mask is not None
        ctx.dg, ctx.H, ctx.agg, ctx.act, ctx.slope, ctx.backend = dg, H, agg, act, slope, backend
        return S

    @staticmethod
    def backward(ctx, dS):
        dg, H, agg, act, slope, backend = ctx.dg, ctx.H, ctx.agg, ctx.act, ctx.slope, ctx.backend
        dev = dS.device
        G = dS.contiguous().float()
        if ctx.masked:
            (mask,) = ctx.saved_tensors
            Q = K_ext = None
        else:
            Q, K_ext = ctx.saved_tensors
            mask = None
        dQ = torch.empty((dg.n_rows, H), device=dev, dtype=torch.float32)
        big, dK_ext, recvs = _backward_buffers(dg, H, dev, torch.float32)
        works = _chunked_backward(backend, dg, H, agg, act, slope, G, Q, K_ext, mask, dQ, dK_ext, recvs)
        dK = _complete_dk(dg, big, recvs, works, backend)
        return dQ, dK, None, None, None, None, None, None, None, None


class HashedDropout(torch.autograd.Function):
    """Feature dropout (conv.py:60-61) with the hashed mask of ``drop`` = (seed, p) (``sir_dropout_apply``:
    keep / scale decided per (local row, column) from the seed); the backward applies the same mask to
    the gradient."""

    @staticmethod
    def forward(ctx, X, drop):
        ctx.drop = drop
        return _native.dropout_apply(X.contiguous().clone(), drop)

    @staticmethod
    def backward(ctx, g):
        return _native.dropout_apply(g.contiguous().clone(), ctx.drop), None


class HaloGather(torch.autograd.Function):
    """K_ext = [K own rows | halo rows of the peers] (forward: the chunked alltoallv); backward: the
    halo rows' gradients go back to their owners (reverse alltoallv) and are added to the own rows per
    chunk and peer in a fixed order (deterministic).  The modular edge-cut route (``agg_type='max'``)."""

    @staticmethod
    def forward(ctx, K, dg):
        n = dg.n_rows
        K_ext = torch.empty((dg.n_ext, K.shape[1]), device=K.device, dtype=K.dtype)
        K_ext[:n] = K
        dg.gather_halo(K_ext[:n], K_ext)
        ctx.dg = dg
        return K_ext

    @staticmethod
    def backward(ctx, dK_ext):
        dg = ctx.dg
        n = dg.n_rows
        dK_ext = dK_ext.contiguous()
        dK = dK_ext[:n].clone()
        for c in range(dg.chunks):
            recv = torch.empty((dg.send_idx[c].numel(), dK.shape[1]), device=dK.device, dtype=dK.dtype)
            dg.scatter_chunk(c, dK_ext, recv)
            dg.add_received(c, dK, recv)
        return dK, None


class DistSIRConv(torch.nn.Module):
    """Wraps a :class:`sirgcn.SIRConv` (same parameters / state_dict) for the edge-cut layout.

    ``forward(dgraph, feat_local)`` takes this rank's rows of X and returns its rows of Y.
    Call :meth:`allreduce_grads` after ``backward`` (data-parallel weight gradients)."""

    use_fused = True

    def __init__(self, conv, backend=None, use_mask=True, reduce_in_backward=False):
        """``reduce_in_backward``: the fused functions all-reduce the weight gradients themselves, dW_R /
        dW_Q under the reverse exchange and dW_K at the end (RCCL, async); :meth:`allreduce_grads`
        then skips what they reduced."""
        super().__init__()
        self.conv = conv
        self.backend = backend if backend is not None else _native
        self.use_mask = use_mask
        self.reduce_in_backward = reduce_in_backward
        self._reduced = False

    def _drop(self, device):
        """(two seeds, p) of this forward's Q / K dropout (conv.py:35,60-61), or None: drawn on the
        device from torch's CUDA generator (graph-safe), on the host for CPU rehearsals."""
        c = self.conv
        if not (c.training and c.dropout.p > 0):
            return None
        if device.type != "cuda":
            return int(torch.randint(0, 2 ** 62, (1,)).item()), float(c.dropout.p)
        return torch.randint(0, 2 ** 62, (2,), device=device, dtype=torch.int64), float(c.dropout.p)

    def forward(self, dgraph, feat):
        c = self.conv
        if c._agg_type not in ("sum", "mean", "sym", "max"):
            raise NotImplementedError(f"DistSIRConv: agg_type={c._agg_type!r}")
        if feat.shape[0] != dgraph.n_rows:
            raise ValueError(f"feat has {feat.shape[0]} rows, rank owns {dgraph.n_rows}")
        act, slope = activation_code(c.activation)
        H = c.linear_query.out_features
        self._reduced = False
        if c._agg_type == "max":
            # conv.py:46-47 + fn.max on the edge-cut: Q, K of the own rows, K's halo rows gathered, then
            # the fused per-edge W_R with the running max (sirgcn.edgemlp) on [own | halo] K rows
            from .edgemlp import EdgeMaxLinearQK, max_supported
            if not (feat.is_cuda and self.backend is _native and max_supported(H, c.linear_relation.out_features)):
                raise NotImplementedError("DistSIRConv max: native GPU path only (H, O <= 512, H % 4 == 0)")
            Q = c._linear(feat, c.linear_query.weight, c.linear_query.bias)
            K = c._linear(feat, c.linear_key.weight, None)
            drop = self._drop(feat.device)
            if drop is not None:
                # the fused paths' hashed masks (seeds mixed with the rank's first global row): local
                # row i of two ranks draws independent bits, as nn.Dropout over the whole [V, H] does
                dq, dk = _drops(drop, dgraph.row_begin)
                Q, K = HashedDropout.apply(Q, dq), HashedDropout.apply(K, dk)
            K_ext = HaloGather.apply(K, dgraph)
            return EdgeMaxLinearQK.apply(Q, K_ext, c.linear_relation.weight, c.linear_relation.bias, dgraph, act, slope)
        # training dropout inside the fused functions needs the native kernels on device tensors (the
        # hashed masks are applied by sir_dropout_apply / the GEMM epilogues): CPU rehearsals and
        # injected edge backends with p > 0 take the modular path (nn.Dropout) instead
        drop_native = feat.is_cuda and self.backend is _native
        fused = (self.use_fused and feat.dtype == torch.float32 and not torch.is_autocast_enabled()
                 and c.linear_query.weight.dtype == torch.float32
                 and (drop_native or not (c.training and c.dropout.p > 0)))
        if fused:
            self._reduced = self.reduce_in_backward
            return DistSIRConvFunction.apply(feat, c.linear_query.weight, c.linear_query.bias, c.linear_key.weight,
                                             c.linear_relation.weight, c.linear_relation.bias, dgraph,
                                             c._agg_type, act, slope, self.backend, self.use_mask,
                                             torch.is_grad_enabled(), self._drop(feat.device), self.reduce_in_backward)
        if (self.use_fused and feat.is_cuda and torch.is_autocast_enabled() and H % 4 == 0
                and c.linear_query.weight.dtype == torch.float32
                and feat.dtype in (torch.float32, torch.bfloat16, torch.float16)):
            dt = torch.get_autocast_dtype("cuda")
            if dt in (torch.bfloat16, torch.float16):
                with torch.autocast("cuda", enabled=False):
                    self._reduced = self.reduce_in_backward
                    return DistSIRConvFunction16.apply(feat, c.linear_query.weight, c.linear_query.bias,
                                                       c.linear_key.weight, c.linear_relation.weight,
                                                       c.linear_relation.bias, dgraph, c._agg_type, act, slope,
                                                       self.backend, self.use_mask, torch.is_grad_enabled(), dt,
                                                       self._drop(feat.device), self.reduce_in_backward)
        Q = c.dropout(c.linear_query(feat))
        K = c.dropout(c.linear_key(feat))
        S = DistEdgeAggregate.apply(Q, K, dgraph, H, c._agg_type, act, slope, self.backend, self.use_mask,
                                    torch.is_grad_enabled())
        return c.linear_relation(S)

    def allreduce_grads(self, group=None):
        if self._reduced:          # the fused backward reduced every weight gradient already
            self._reduced = False
            return
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

"""Fused per-edge dense layer (``sir_edge_mlp_*``, csrc/sirconv_edgemlp.hip): the two SIRConv forms
whose message runs a Linear on every edge, without any [E, *] tensor in the forward.

* ``Sequential(act1, Linear(H, F), act2)`` sigma (``dictionary-lookup/model.py:17``, used through
  ``conv.py:45``) with sum / mean / sym: :class:`EdgeMLPSum` — forward and backward fused for
  H, F <= 256 (the config-1 shape is H = F = 64; the DictionaryLookup sweep reaches H = F = 200,
  ``dictionary-lookup/README.md:8``).
* ``agg_type='max'`` (``conv.py:46-47``: ``linear_relation`` per edge, DGL ``fn.max``):
  :class:`EdgeMaxLinear` — fused forward (running max with the first arg-max edge) and four
  backwards: the hybrid one by default where its routing table fits the memory budget (H <= 512,
  O <= 256: dQ / dK from the routed passes of ``sir_edge_max_bwd_sparse`` — the (v, o) pairs grouped by
  their arg edge, dA_e from the W_R rows of e's routed outputs only, V O H multiply-adds per product
  instead of E O H — and dW_R / db_R from ``sir_max_dw_qk`` with the activations recomputed per row
  batch: no [E, *] tensor); the edge-materialised one otherwise (edge activations recomputed once into
  [E, H] buffers, native gather / split-fp16 GEMM / segment kernels, over destination-row ranges past
  the budget); the fully routed one (opt-in ``sparse_bwd``: dW_R from a_{arg} per (v, o)); the dense
  fused one (fp32 MFMA, opt-in ``fused_bwd``).

Under autocast (the reference trains its max configs with AMP, ``heterophilous-datasets/train.py:75``)
the max forward reads Q, K in their 16-bit storage and runs the per-edge Linear as the reference's
half-precision nn.Linear does: a = act1(Q[v] + K[u]) evaluated in fp32 and rounded once to the 16-bit type,
h = a W^T + b as one 16-bit MFMA per 16 k on W, b rounded to it, fp32 accumulation
(``sir_edge_mlp_fwd*_st``, round 6); the max and its arg edge are taken over the fp32 h (the reference
rounds h to 16 bits first: its ties among equal rounded values may pick another edge).  The max backward
and the Sequential-sigma form widen Q, K to fp32 (a V-sized copy) and run the fp32 kernels — more accurate
than the reference's 16-bit backward, not bit-level AMP parity (the reference trains only its max and
sym configs under AMP, ``heterophilous-datasets/train.py:191-223``; the Sequential sigma's
DictionaryLookup runs in fp32) (``tests/test_amp_gpu.py::
test_fused_edge_mlp_forms_under_autocast``).  A CPU tensor or a shape outside the kernels' limits is
never silently served by another path — :func:`seq_sigma` / :func:`max_supported` say up front which
form applies.
"""
import ctypes

import warnings

import torch
from torch import nn
import torch.nn.functional as F

from . import _native, linalg

AGG_MAX = 3


def _elementwise_code(m):
    """Kernel code of an elementwise activation module (None if not one of the kernel's)."""
    if isinstance(m, nn.LeakyReLU):
        return _native.ACT_LEAKY, float(m.negative_slope)
    if isinstance(m, nn.ReLU):
        return _native.ACT_RELU, 0.0
    if isinstance(m, nn.GELU):
        return (_native.ACT_GELU_TANH if m.approximate == "tanh" else _native.ACT_GELU), 0.0
    if isinstance(m, nn.Identity):
        return _native.ACT_IDENTITY, 0.0
    return None


def seq_sigma(act, H):
    """(act1, slope, linear, act2) when ``act`` is Sequential(elementwise, Linear(H, F), ReLU|Identity)
    within the fused kernels' limits, else None."""
    if not isinstance(act, nn.Sequential) or len(act) != 3:
        return None
    a1, lin, a2 = act[0], act[1], act[2]
    c1 = _elementwise_code(a1)
    c2 = _elementwise_code(a2)
    if c1 is None or c2 is None or c2[0] not in (_native.ACT_RELU, _native.ACT_IDENTITY):
        return None
    if not isinstance(lin, nn.Linear) or lin.in_features != H or H % 4 or H > 256 or lin.out_features > 256:
        return None
    return c1[0], c1[1], lin, c2[0]


def max_supported(H, O):
    """The max form's fused forward: H, O <= 512 (roman-empire's H = O = 512,
    heterophilous-datasets/README.md:8)."""
    return H % 4 == 0 and H <= 512 and O <= 512


def _pack(W):
    lib = _native.load()
    Fo, H = W.shape
    nbytes = lib.sir_edge_mlp_pack_bytes(H, Fo)
    packed = torch.empty((nbytes,), dtype=torch.uint8, device=W.device)
    rc = lib.sir_edge_mlp_pack(_native._ptr(W), H, Fo, _native._ptr(packed), _native._stream(W.device))
    _native._check(rc, lib)
    return packed


# the edge-stream forward (sir_edge_mlp_fwd_stream) for H = 256, F <= 256; False: the per-item kernels
STREAM = True


def _edge_rows(csr):
    """Destination row of every dst-CSR edge (int32, cached on the plan)."""
    er = getattr(csr, "_erow", None)
    if er is None:
        deg = (csr.rowptr[1:] - csr.rowptr[:-1]).long()
        er = torch.repeat_interleave(torch.arange(csr.n_rows, device=deg.device, dtype=torch.int32), deg)
        csr._erow = er
    return er


# 16-bit Q / K (autocast) on the max forward's 16-bit kernels; False: widened to fp32 (the fp32 kernels)
NATIVE_16 = True


def _st_ok(QK, H):
    return (NATIVE_16 and QK.dtype in (torch.bfloat16, torch.float16) and QK.dim() == 2 and QK.stride(1) == 1
            and QK.stride(0) % 4 == 0 and H % 4 == 0 and QK.data_ptr() % 8 == 0)


def _fwd_st(plan, Q, K, W, b, act1, slope, out, arg):
    """The max forward on 16-bit Q, K rows (``sir_edge_mlp_pack_st`` + ``sir_edge_mlp_fwd_stream_st`` /
    ``sir_edge_mlp_fwd_st``): one 16-bit MFMA per product, fp32 accumulation, fp32 ``out``."""
    lib = _native.load()
    csr = plan.dst
    Fo, H = W.shape
    dt = _native.STORAGE[Q.dtype]
    P = _native._ptr
    st = _native._stream(Q.device)
    packed = torch.empty((lib.sir_edge_mlp_pack_bytes(H, Fo),), dtype=torch.uint8, device=Q.device)
    _native._check(lib.sir_edge_mlp_pack_st(P(W), H, Fo, dt, P(packed), st), lib)
    if STREAM and H == 256 and Fo <= 256:
        E = csr.col.numel()
        work = torch.empty((lib.sir_edge_mlp_stream_work_bytes(Fo),), dtype=torch.uint8, device=Q.device)
        with _native._Timed("sir_edge_mlp_fwd", Q.device, 2 * E * H * Fo):
            rc = lib.sir_edge_mlp_fwd_stream_st(P(csr.rowptr), P(csr.col) if E else None,
                                                P(_edge_rows(csr)) if E else None, csr.n_rows, E, H, Fo, P(Q),
                                                Q.stride(0), P(K), K.stride(0), dt, AGG_MAX, act1, float(slope),
                                                _native.ACT_IDENTITY, P(packed), P(b), P(out), out.stride(0), P(arg),
                                                arg.stride(0), P(work), st)
        _native._check(rc, lib)
        return
    n = csr.n_slots
    pval = torch.empty((max(n, 1) * Fo,), device=Q.device, dtype=torch.float32) if n else None
    parg = torch.empty((max(n, 1) * Fo,), device=Q.device, dtype=torch.int32) if n else None
    with _native._Timed("sir_edge_mlp_fwd", Q.device, 2 * csr.col.numel() * H * Fo):
        rc = lib.sir_edge_mlp_fwd_st(P(csr.rowptr), P(csr.col), P(csr.items), csr.n_items, P(csr.splits),
                                     csr.n_splits, H, Fo, P(Q), Q.stride(0), P(K), K.stride(0), dt, AGG_MAX, act1,
                                     float(slope), _native.ACT_IDENTITY, P(packed), P(b), P(out), out.stride(0),
                                     P(arg), arg.stride(0), P(pval), P(parg), st)
    _native._check(rc, lib)


def _fwd(plan, Q, K, W, b, agg, act1, slope, act2, out, arg=None):
    lib = _native.load()
    csr = plan.dst
    Fo, H = W.shape
    in_norm, out_norm = plan.norms(agg if agg != "max" else "sum")
    packed = _pack(W)
    P = _native._ptr
    if STREAM and H == 256 and Fo <= 256:
        E = csr.col.numel()
        work = torch.empty((lib.sir_edge_mlp_stream_work_bytes(Fo),), dtype=torch.uint8, device=Q.device)
        code = AGG_MAX if agg == "max" else _native.AGG[agg]
        with _native._Timed("sir_edge_mlp_fwd", Q.device, 2 * E * H * Fo):
            rc = lib.sir_edge_mlp_fwd_stream(P(csr.rowptr), P(csr.col) if E else None, P(_edge_rows(csr)) if E else None,
                                             csr.n_rows, E, H, Fo, P(Q), Q.stride(0), P(K), K.stride(0), P(in_norm),
                                             P(out_norm), code, act1, float(slope), act2, P(packed), P(b), P(out),
                                             out.stride(0), P(arg), arg.stride(0) if arg is not None else Fo, P(work),
                                             _native._stream(Q.device))
        _native._check(rc, lib)
        return packed
    n = csr.n_slots
    pval = torch.empty((max(n, 1) * Fo,), device=Q.device, dtype=torch.float32) if n else None
    parg = torch.empty((max(n, 1) * Fo,), device=Q.device, dtype=torch.int32) if (n and arg is not None) else None
    code = AGG_MAX if agg == "max" else _native.AGG[agg]
    with _native._Timed("sir_edge_mlp_fwd", Q.device, 2 * csr.col.numel() * H * Fo):
        rc = lib.sir_edge_mlp_fwd(P(csr.rowptr), P(csr.col), P(csr.items), csr.n_items, P(csr.splits), csr.n_splits,
                                  H, Fo, P(Q), Q.stride(0), P(K), K.stride(0), P(in_norm), P(out_norm), code, act1,
                                  float(slope), act2, P(packed), P(b), P(out), out.stride(0), P(arg),
                                  arg.stride(0) if arg is not None else Fo, P(pval), P(parg), _native._stream(Q.device))
    _native._check(rc, lib)
    return packed


class EdgeMLPSum(torch.autograd.Function):
    """S[v] = sum_e c_e act2(W act1(Q[v] + K[u]) + b) (mean: / deg) for QK = [Q | K]."""

    @staticmethod
    def forward(ctx, QK, W, b, plan, H, agg, act1, slope, act2):
        if QK.device.type != "cuda":
            raise RuntimeError("sirgcn fused edge MLP needs a ROCm GPU tensor (no CPU fallback)")
        QK = QK.contiguous().float()
        W = W.contiguous().float()
        b = b.contiguous().float() if b is not None else None
        Fo = W.shape[0]
        S = torch.empty((plan.dst.n_rows, Fo), device=QK.device, dtype=torch.float32)
        packed = _fwd(plan, QK[:, :H], QK[:, H:], W, b, agg, act1, slope, act2, S)
        ctx.save_for_backward(QK, W, b if b is not None else W.new_zeros(0), packed)
        ctx.plan, ctx.H, ctx.agg, ctx.act1, ctx.slope, ctx.act2, ctx.has_b = plan, H, agg, act1, slope, act2, b is not None
        return S

    @staticmethod
    def backward(ctx, dS):
        QK, W, b, packed = ctx.saved_tensors
        plan, H, agg, act1, slope, act2 = ctx.plan, ctx.H, ctx.agg, ctx.act1, ctx.slope, ctx.act2
        lib = _native.load()
        P = _native._ptr
        G = dS.contiguous().float()
        Fo = W.shape[0]
        dev = G.device
        bias = b if ctx.has_b else None
        in_norm, out_norm = plan.norms(agg)
        Q, K = QK[:, :H], QK[:, H:]
        dQK = torch.empty_like(QK)
        d, s = plan.dst, plan.src
        waves = lib.sir_edge_mlp_bwd_parts(d.n_items, H, Fo)
        FP, HP = (Fo + 31) // 32 * 32, (H + 7) // 8 * 8
        wpart = torch.empty((waves, FP * HP + FP), device=dev, dtype=torch.float32)
        part = torch.empty((max(d.n_slots, s.n_slots, 1) * H,), device=dev, dtype=torch.float32)
        Gm = torch.empty((d.n_rows, Fo), device=dev, dtype=torch.float32) if agg == "mean" else None
        st = _native._stream(dev)
        code = _native.AGG[agg]
        with _native._Timed("sir_edge_mlp_bwd_dst", dev):
            rc = lib.sir_edge_mlp_bwd_dst(P(d.rowptr), P(d.col), P(d.items), d.n_items, P(d.splits), d.n_splits, H, Fo,
                                          P(Q), Q.stride(0), P(K), K.stride(0), P(G), G.stride(0), P(in_norm),
                                          P(out_norm), code, act1, float(slope), act2, P(packed), P(W), P(bias),
                                          P(dQK), dQK.stride(0), P(Gm), P(part), P(wpart), st)
        _native._check(rc, lib)
        Gd = Gm if Gm is not None else G
        with _native._Timed("sir_edge_mlp_bwd_src", dev):
            rc = lib.sir_edge_mlp_bwd_src(P(s.rowptr), P(s.col), P(s.items), s.n_items, P(s.splits), s.n_splits, H, Fo,
                                          P(K), K.stride(0), P(Q), Q.stride(0), P(Gd), Gd.stride(0), P(out_norm),
                                          P(in_norm), code, act1, float(slope), act2, P(packed), P(W), P(bias),
                                          P(dQK[:, H:]), dQK.stride(0), P(part), st)
        _native._check(rc, lib)
        tot = _native.col_sum(wpart)                    # per-wave partials summed in wave order
        dW = tot[:FP * HP].view(FP, HP)[:Fo, :H].contiguous()
        db = tot[FP * HP:FP * HP + Fo].contiguous() if ctx.has_b else None
        return dQK, dW, db, None, None, None, None, None, None


class EdgeMaxLinear(torch.autograd.Function):
    """Y[v] = max_e (W_R act1(Q[v] + K[u]) + b_R), first arg-max edge (DGL fn.max), empty rows 0.

    Backward route (``fused_bwd``): ``None`` (default) — with ``sparse_bwd`` the routed backward
    (``max_bwd_sparse``: H % 4 == 0, H <= 512, O <= 256; no [E, *] buffer, V O H multiply-adds per product),
    else the edge-materialised one (z recomputed once into [E, H], dM [E, O]; its GEMMs on the split-fp16
    MFMA kernels), over the whole
    graph when its buffers, E (2H + O) 4 bytes, stay within ``materialised_budget`` (48 GiB, and 40 % of
    the free device memory), else over destination-row ranges that each fit it; ``True`` — the fused
    backward (no [E, *] buffer; its three edge-contracted products on fp32 MFMA, 14x slower at S2);
    ``False`` — the materialised one (tests)."""
    fused_bwd = None
    # True: the routed backward (no [E, *] buffer) for H % 4 == 0, H <= 512, O <= 256 when fused_bwd is None.
    # Off by default: its dW_R pass (a_{arg} gathered per (v, o), L1-bound) makes it slower than the
    # edge-materialised route at S1 / S2 (36.0 vs 30.4 ms S1 max step, 138 vs 120 ms S2 max)
    sparse_bwd = False
    # True: A [E, H] materialised for dW_R (sir_max_dw_rows), dQ / dK from the routed passes (no dM, no dZ)
    hybrid_bwd = True
    dw_qk = True                # hybrid route: dW_R from Q, K recomputed per row batch (no A buffer)
    dw_rows = True              # materialised route: dW_R / db_R from A and the arg edges (sir_max_dw_rows)
    materialised_budget = 48 << 30

    @staticmethod
    def forward(ctx, QK, W, b, plan, H, act1, slope):
        if QK.device.type != "cuda":
            raise RuntimeError("sirgcn fused max path needs a ROCm GPU tensor (no CPU fallback)")
        W = W.contiguous().float()
        b = b.contiguous().float() if b is not None else None
        O = W.shape[0]
        V = plan.dst.n_rows
        Y = torch.empty((V, O), device=QK.device, dtype=torch.float32)
        arg = torch.empty((V, O), device=QK.device, dtype=torch.int32)
        if _st_ok(QK, H):             # autocast: 16-bit rows, 16-bit per-edge Linear (module docstring)
            _fwd_st(plan, QK[:, :H], QK[:, H:], W, b, act1, slope, Y, arg)
        else:
            QK = QK.contiguous().float()
            _fwd(plan, QK[:, :H], QK[:, H:], W, b, "max", act1, slope, _native.ACT_IDENTITY, Y, arg)
        ctx.save_for_backward(QK, W, arg)
        ctx.plan, ctx.H, ctx.act1, ctx.slope, ctx.has_b = plan, H, act1, slope, b is not None
        return Y

    @staticmethod
    def backward(ctx, dY):
        QK, W, arg = ctx.saved_tensors
        H = ctx.H
        QK = QK.float()               # 16-bit rows of the autocast forward: the fp32 backward on widened rows
        dQK = torch.empty_like(QK)
        dW, db = max_linear_backward(ctx.plan, QK[:, :H], QK[:, H:], W, arg, dY, ctx.act1, ctx.slope,
                                     dQK[:, :H], dQK[:, H:])
        return dQK, dW, (db if ctx.has_b else None), None, None, None, None


class EdgeMaxLinearQK(torch.autograd.Function):
    """:class:`EdgeMaxLinear` on separate Q [dst rows, H] and K [src rows, H] (the edge-cut's own-row Q
    and K_ext = own + halo rows, sirgcn.dist): the plan's dst CSR columns index K, its src CSR rows
    are K's rows.  Same kernels, same backward routes."""

    @staticmethod
    def forward(ctx, Q, K, W, b, plan, act1, slope):
        if Q.device.type != "cuda":
            raise RuntimeError("sirgcn fused max path needs a ROCm GPU tensor (no CPU fallback)")
        Q, K = Q.contiguous().float(), K.contiguous().float()
        W = W.contiguous().float()
        b = b.contiguous().float() if b is not None else None
        O = W.shape[0]
        V = plan.dst.n_rows
        Y = torch.empty((V, O), device=Q.device, dtype=torch.float32)
        arg = torch.empty((V, O), device=Q.device, dtype=torch.int32)
        _fwd(plan, Q, K, W, b, "max", act1, slope, _native.ACT_IDENTITY, Y, arg)
        ctx.save_for_backward(Q, K, W, arg)
        ctx.plan, ctx.act1, ctx.slope, ctx.has_b = plan, act1, slope, b is not None
        return Y

    @staticmethod
    def backward(ctx, dY):
        Q, K, W, arg = ctx.saved_tensors
        dQ, dK = torch.empty_like(Q), torch.empty_like(K)
        dW, db = max_linear_backward(ctx.plan, Q, K, W, arg, dY, ctx.act1, ctx.slope, dQ, dK)
        return dQ, dK, dW, (db if ctx.has_b else None), None, None, None


def max_linear_backward(plan, Q, K, W, arg, dY, act1, slope, dQ, dK):
    """Backward of Y[v] = max_e (W act1(Q[v] + K[u]) + b): dQ / dK written into the given views,
    returns (dW, db).  Route by ``EdgeMaxLinear.fused_bwd`` (see there)."""
    H = Q.shape[1]
    dY = dY.contiguous().float()
    O = W.shape[0]
    E = plan.dst.col.numel()
    dev = dY.device
    fused = EdgeMaxLinear.fused_bwd
    if fused and max_bwd_fused(H, O):
        return _max_bwd_fused(plan, Q, K, W, arg, dY, H, act1, slope, dQ, dK)
    if fused is None and EdgeMaxLinear.sparse_bwd and max_bwd_sparse(H, O, plan.dst.n_rows):
        return _max_bwd_sparse(plan, Q, K, W, arg, dY, act1, slope, dQ, dK)
    per_edge = (2 * H + O) * 4
    # free device memory as the caching allocator sees it: the driver's free bytes plus the blocks it
    # has reserved but not handed out (a warm training loop holds most memory there)
    avail = torch.cuda.mem_get_info(dev)[0] + torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    budget = min(EdgeMaxLinear.materialised_budget, int(0.4 * avail))
    V = plan.dst.n_rows
    # the hybrid's buffers: the routing table (16 B per edge, 8 per (v, o)) and, without dw_qk, A [E, H]
    hyb = E * (16 + (0 if EdgeMaxLinear.dw_qk else 4 * H)) + V * O * 8
    if fused is None and EdgeMaxLinear.hybrid_bwd and max_bwd_sparse(H, O, V) and hyb <= budget:
        return _max_bwd_hybrid(plan, Q, K, W, arg, dY, act1, slope, dQ, dK)
    if E * per_edge > budget and E > 0:
        # the [E, *] buffers exceed the budget: the same dataflow over destination-row ranges of
        # <= budget / per_edge edges each (the S2 shape: 123 GB of buffers -> 3 ranges of <= 48 GiB)
        # range size quantised (a stable cache key while the free memory moves): to 4 Mi edges, below
        # that to a power of two that still fits, at least 4 Ki edges (past the budget only then: warned)
        e_fit = max(int(budget) // per_edge, 0)
        e_max = e_fit >> 22 << 22 if e_fit >= 1 << 22 else 1 << max(e_fit.bit_length() - 1, 12)
        if e_max > e_fit:
            warnings.warn(f"max backward: {e_max} edges per row range need {e_max * per_edge / 2**30:.2f} GiB, "
                          f"past the {budget / 2**30:.2f} GiB budget", RuntimeWarning)
        return _max_bwd_ranges(plan, Q, K, W, arg, dY, act1, slope, dQ, dK, e_max)
    return _max_bwd_materialised(plan.dst, plan.src, Q, K, W, arg, dY, act1, slope, dQ, dK)


def _max_bwd_ranges(plan, Q, K, W, arg, dY, act1, slope, dQ, dK, e_max):
    """The edge-materialised max backward over destination-row ranges of <= e_max edges: each range is
    its own sub-graph (rows rebased to 0, its edges in dst-CSR order, a source-side CSR over all K rows;
    built once per plan and cached), dW_R / db_R summed over the ranges in order, dK accumulated
    over the ranges in order (deterministic)."""
    key = ("max_ranges", int(e_max))
    cache = getattr(plan, "_sub_plans", None)
    if cache is None:
        cache = plan._sub_plans = {}
    if key not in cache:
        cache[key] = _row_ranges(plan.dst, K.shape[0], int(e_max))
    dW = db = None
    first = True
    for r0, r1, e0, d_c, s_c in cache[key]:
        dK_c = dK if first else torch.empty_like(dK)
        a_c = arg[r0:r1] - e0 if e0 else arg[r0:r1]                # arg edges as positions inside the range
        w, b = _max_bwd_materialised(d_c, s_c, Q[r0:r1], K, W, a_c, dY[r0:r1], act1, slope, dQ[r0:r1], dK_c)
        if first:
            dW, db = w, b
        else:
            dW += w
            db += b
            dK += dK_c
        first = False
    return dW, db


def _row_ranges(dst, n_src, e_max):
    """[(r0, r1, e0, dst sub-CSR, src sub-CSR)] of consecutive destination rows holding <= e_max edges
    (a row longer than e_max gets a range of its own)."""
    from .graph import build_plans_native
    rp = dst.rowptr.to(torch.int64).cpu()
    n = rp.numel() - 1
    out, r0 = [], 0
    while r0 < n:
        e0 = int(rp[r0])
        r1 = int(torch.searchsorted(rp, torch.tensor(e0 + e_max), right=True)) - 1
        r1 = min(max(r1, r0 + 1), n)
        e1 = int(rp[r1])
        deg = (dst.rowptr[r0 + 1:r1 + 1] - dst.rowptr[r0:r1]).to(torch.int64)
        rows = torch.repeat_interleave(torch.arange(r1 - r0, device=deg.device), deg)
        d_c, s_c = build_plans_native(dst.col[e0:e1].to(torch.int64), rows, r1 - r0, n_src)
        out.append((r0, r1, e0, d_c, s_c))
        r0 = r1
    return out


def _max_bwd_materialised(dcsr, scsr, Q, K, W, arg, dY, act1, slope, dQ, dK):
    """The edge-materialised max backward over one (sub-)graph: z recomputed once into [E, H], dM = dY
    routed to the first arg-max edges [E, O], dW_R = dM^T A and dZ = sigma'(z) (dM W_R) on the split-fp16
    GEMMs, dQ / dK by native segment sums.  Returns (dW, db)."""
    H = Q.shape[1]
    O = W.shape[0]
    E = dcsr.col.numel()
    dev = dY.device
    dY = dY.contiguous()
    # the arg edges' activations are needed for dW_R: recompute them once (no copy kept from the
    # forward).  ReLU family: A = sigma(z) straight from the gather (sign(A) = sign(z), so sigma' is
    # read off A below and z is never stored); other sigmas: z, then sigma(z).  A LeakyReLU with a
    # negative slope flips the sign (z < 0 gives A = slope z > 0), so it takes the z route
    relu_family = act1 == _native.ACT_RELU or (act1 == _native.ACT_LEAKY and slope >= 0)
    smask = None
    if relu_family:
        A = torch.empty((E, H), device=dev, dtype=torch.float32)
        if H == 256:            # sign words for the gated GEMM: 32 B per edge instead of A's 1 KiB
            smask = torch.empty((E, 4), device=dev, dtype=torch.int64)
        _native.edge_gather_act(dcsr, Q, K, act1, slope, A, sign_mask=smask)
        Z = A
    else:
        Z = torch.empty((E, H), device=dev, dtype=torch.float32)
        _native.edge_gather_add(dcsr, Q, K, Z)
        A = _act(Z, act1, slope)
    dM = torch.empty((E, O), device=dev, dtype=torch.float32)
    _native.segment_max_bwd(dcsr, arg, dY, dM)                     # dY to the first arg-max edge
    if EdgeMaxLinear.dw_rows and O <= 256 and H % 4 == 0 and A.is_contiguous():
        # dW_R[o] = sum_v dY[v][o] A[arg[v][o]]: each row's A rows read once, V O H multiply-adds
        dW, db = _native.max_dw_rows(dcsr, arg, dY, A, O)
    else:
        dW, db = linalg.mm_tn(dM, A, colsum=True)                  # dW_R = dM^T A, db_R = sum dM
    if relu_family:     # dZ = sigma'(z) * (dM W_R) with sigma' read off A in the GEMM's epilogue
        dZ = linalg.mm_w_dact(dM, W, A, act1, slope, gate_mask=smask)
        del A, Z, dM
    else:
        del A
        dA = linalg.mm_w(dM, W)                                    # [E, H]
        del dM
        dZ = _act_bwd(Z, dA, act1, slope)
        del Z, dA
    n_slots = max(dcsr.n_slots, scsr.n_slots)
    part = torch.empty((max(n_slots, 1) * H,), device=dev, dtype=torch.float32) if n_slots else None
    _native.segment_sum(dcsr, dZ, dQ, partial=part)                     # dQ
    _native.segment_sum(scsr, dZ, dK, perm=scsr.perm, partial=part)     # dK
    return dW, db


def max_bwd_sparse(H, O, V):
    """The routed backward (``sir_edge_max_bwd_sparse``) covers H % 4 == 0, H <= 512, O <= 256."""
    return H % 4 == 0 and 0 < H <= 512 and 0 < O <= 256 and V * O < 2 ** 31 - 1


def _max_bwd_hybrid(plan, Q, K, W, arg, dY, act1, slope, dQ, dK):
    """A = act1(z) materialised once ([E, H], dst-CSR order) for dW_R / db_R (``sir_max_dw_rows``); dQ / dK
    from the routed passes (``sir_edge_max_bwd_sparse`` without its dW pass): no dM [E, O], no dZ [E, H]."""
    H, O = Q.shape[1], W.shape[0]
    d = plan.dst
    E = d.col.numel()
    dev = dY.device
    if EdgeMaxLinear.dw_qk:
        # dW_R with the activations recomputed per row batch: no [E, *] buffer anywhere in the backward
        _max_bwd_sparse(plan, Q, K, W, arg, dY, act1, slope, dQ, dK, with_dw=False)
        return _native.max_dw_qk(d, arg, dY, Q, K, O, act1, slope)
    A = torch.empty((max(E, 1), H), device=dev, dtype=torch.float32)[:E]
    if act1 in (_native.ACT_RELU, _native.ACT_LEAKY, _native.ACT_IDENTITY):
        _native.edge_gather_act(d, Q, K, act1, slope, A)
    else:
        _native.edge_gather_add(d, Q, K, A)
        A = _act(A, act1, slope)
    _max_bwd_sparse(plan, Q, K, W, arg, dY, act1, slope, dQ, dK, with_dw=False)
    return _native.max_dw_rows(d, arg, dY, A, O)


def _src_pinv(plan):
    """dst-CSR position -> src-CSR position (the inverse of the source CSR's perm), cached on the plan."""
    pinv = getattr(plan, "_pinv", None)
    if pinv is None:
        perm = plan.src.perm
        pinv = torch.empty_like(perm)
        pinv[perm.long()] = torch.arange(perm.numel(), device=perm.device, dtype=perm.dtype)
        plan._pinv = pinv
    return pinv


def _max_bwd_sparse(plan, Q, K, W, arg, dY, act1, slope, dQ, dK, with_dw=True):
    """``sir_edge_max_bwd_sparse``: the (v, o) pairs grouped by their arg edge (a routing table of
    8 V O + 16 E bytes), dA_e from the |L_e| W_R rows its routed outputs name, dQ / dK by row passes of
    both CSRs, dW_R from a_{arg} gathered per (v, o) — V O H multiply-adds per product, no [E, *] buffer."""
    lib = _native.load()
    P = _native._ptr
    H, O = Q.shape[1], W.shape[0]
    d, s = plan.dst, plan.src
    V, E = d.n_rows, d.col.numel()
    dev = dY.device
    W = W.contiguous()
    rb, nr = ctypes.c_int64(0), ctypes.c_int64(0)
    _native._check(lib.sir_edge_max_bwd_sparse_parts(d.n_items, V, ctypes.byref(rb), ctypes.byref(nr)), lib)
    ent = torch.empty((V * O + 8,), device=dev, dtype=torch.int64)     # + the dz passes' queue counters
    ecnt_d = torch.empty((max(E, 1),), device=dev, dtype=torch.int64)
    ecnt_s = torch.empty((max(E, 1),), device=dev, dtype=torch.int64)
    part = torch.empty((max(d.n_slots, s.n_slots, 1) * H,), device=dev, dtype=torch.float32)
    dbpart = torch.empty((rb.value, (O + 3) // 4 * 4), device=dev, dtype=torch.float32)
    wpart = torch.empty((nr.value, O * H), device=dev, dtype=torch.float32) if with_dw else None
    pinv = _src_pinv(plan) if E else None
    with _native._Timed("sir_edge_max_bwd_sparse", dev):
        rc = lib.sir_edge_max_bwd_sparse(P(d.rowptr), P(d.col), P(d.items), d.n_items, P(d.splits), d.n_splits,
                                         P(s.col), P(s.items), s.n_items, P(s.splits), s.n_splits, P(pinv), V, E,
                                         H, O, P(Q), Q.stride(0), P(K), K.stride(0), P(dY), dY.stride(0), P(arg),
                                         arg.stride(0), act1, float(slope), P(W), P(dQ), dQ.stride(0), P(dK),
                                         dK.stride(0), P(part), P(ent), P(ecnt_d), P(ecnt_s), P(dbpart), P(wpart),
                                         _native._stream(dev))
    _native._check(rc, lib)
    if not with_dw:
        return None, None
    db = _native.col_sum(dbpart)[:O]                # per-block partials summed in block order
    dW = _native.col_sum(wpart).view(O, H)          # per-range partials summed in range order
    return dW, db


def max_bwd_fused(H, O):
    """The max form's backward runs fused (no [E, *] tensor) for H, O <= 256."""
    return H % 4 == 0 and H <= 256 and O <= 256


def _max_bwd_fused(plan, Q, K, W, arg, dY, H, act1, slope, dQ, dK):
    """``sir_edge_max_bwd_dst`` (dQ, per-block dW_R / db_R partials) + ``sir_edge_max_bwd_src`` (dK):
    dY reaches each (v, o)'s first arg-max edge only; z, a recomputed per edge."""
    lib = _native.load()
    P = _native._ptr
    O = W.shape[0]
    dev = dY.device
    d, s = plan.dst, plan.src
    parts = lib.sir_edge_mlp_bwd_parts(d.n_items, H, O)
    OP, HP = (O + 31) // 32 * 32, (H + 7) // 8 * 8
    wpart = torch.empty((parts, OP * HP + OP), device=dev, dtype=torch.float32)
    part = torch.empty((max(d.n_slots, s.n_slots, 1) * H,), device=dev, dtype=torch.float32)
    st = _native._stream(dev)
    with _native._Timed("sir_edge_max_bwd_dst", dev):
        rc = lib.sir_edge_max_bwd_dst(P(d.rowptr), P(d.col), P(d.items), d.n_items, P(d.splits), d.n_splits, H, O,
                                      P(Q), Q.stride(0), P(K), K.stride(0), P(dY), dY.stride(0), P(arg),
                                      arg.stride(0), act1, float(slope), P(W), P(dQ), dQ.stride(0), P(part),
                                      P(wpart), st)
    _native._check(rc, lib)
    with _native._Timed("sir_edge_max_bwd_src", dev):
        rc = lib.sir_edge_max_bwd_src(P(s.rowptr), P(s.col), P(s.perm), P(s.items), s.n_items, P(s.splits),
                                      s.n_splits, H, O, P(K), K.stride(0), P(Q), Q.stride(0), P(dY), dY.stride(0),
                                      P(arg), arg.stride(0), act1, float(slope), P(W), P(dK), dK.stride(0),
                                      P(part), st)
    _native._check(rc, lib)
    tot = _native.col_sum(wpart)                    # per-block partials summed in block order
    dW = tot[:OP * HP].view(OP, HP)[:O, :H].contiguous()
    db = tot[OP * HP:OP * HP + O].contiguous()
    return dW, db


def _act(z, code, slope):
    if code == _native.ACT_RELU:
        return torch.relu(z)
    if code == _native.ACT_LEAKY:
        return F.leaky_relu(z, slope)
    if code == _native.ACT_GELU:
        return F.gelu(z)
    if code == _native.ACT_GELU_TANH:
        return F.gelu(z, approximate="tanh")
    return z.clone()


def _act_bwd(z, g, code, slope, is_result=False):
    """sigma'(z) * g with torch's own backward kernels (the ops autograd runs: one fused pass over
    the [E, H] tensors instead of compare + multiply + select, ~3x fewer bytes).  ``is_result``: ``z``
    holds sigma(z) (ReLU family: the same sign, so the same sigma'), computed in place into ``g``."""
    if code == _native.ACT_RELU:
        return torch.ops.aten.threshold_backward(g, z, 0.0)
    if code == _native.ACT_LEAKY:
        return torch.ops.aten.leaky_relu_backward(g, z, slope, is_result)
    if code in (_native.ACT_GELU, _native.ACT_GELU_TANH):
        zz = z.detach().requires_grad_(True)
        with torch.enable_grad():
            y = _act(zz, code, slope)
            (r,) = torch.autograd.grad(y, zz, g)
        return r
    return g

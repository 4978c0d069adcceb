"""CPU restatement of the reference SIRConv layer (TEST INFRASTRUCTURE ONLY).

Reference: briangodwinlim/SIR-GCN ``models/conv.py:7-67`` (snapshot 2025-08-24), whose sparse
part runs inside DGL 2.1.0 (absent; its behaviour is restated from its published source, see
``tests/golden/dgl_shim``).  Each function cites the reference line it follows.

Two flavours live here:

* kernel-level functions (``edge_agg_fwd`` / ``edge_agg_bwd``) that compute exactly what the
  HIP edge kernels compute, given Q, K, dS -> S, dQ, dK; used by the GPU parity tests;
* ``reference_cpu_step`` — the reference's CPU dataflow (DGL edge-UDF path: ``index_select``
  gathers -> add -> sigma -> norm product -> ``index_add`` -> W_R) with torch autograd for the
  backward; this is the ``cpu_baseline`` timed by ``bench.py`` ("port") and the whole-layer
  checker (``layer_fwd_bwd``).

Everything is torch-CPU (or numpy for the integer CSR work); no GPU, no product imports.
"""
import math

import numpy as np
import torch

AGGS = ("sum", "mean", "sym")
ACTS = ("identity", "relu", "leaky", "gelu", "gelu_tanh")


# ----------------------------------------------------------------------------- graph
def csr_by_dst(src, dst, num_nodes):
    """In-edge CSR (DGL's CSC): rows = dst, ``col`` = src, ``eid`` ascending inside a row.

    [DGL-ext] DGL builds CSC by a stable sort of COO by dst (edge-id order kept), which is
    the order ``SpMMSumCsr`` accumulates in (``conv.py:63`` -> gspmm).  Bit-exact target.
    """
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    eid = np.argsort(dst, kind="stable").astype(np.int64)
    counts = np.bincount(dst, minlength=num_nodes).astype(np.int64)
    rowptr = np.zeros(num_nodes + 1, dtype=np.int64)
    np.cumsum(counts, out=rowptr[1:])
    return rowptr, src[eid], eid


def csr_by_src(src, dst, num_nodes):
    """Out-edge CSR: rows = src, ``col`` = dst, ``eid`` ascending (autograd of the src
    gather, ``index_add`` in edge order, accumulates dK[u] in exactly this order)."""
    return csr_by_dst(dst, src, num_nodes)


def degree_norms(in_deg, out_deg, agg):
    """``conv.py:51-57``: clamp(min=1) float degrees; ``sym`` -> deg^-0.5 else ones; fp32."""
    in_degs = torch.as_tensor(in_deg).float().clamp(min=1)
    out_degs = torch.as_tensor(out_deg).float().clamp(min=1)
    n = in_degs.numel()
    in_norm = torch.pow(in_degs, -0.5) if agg == "sym" else torch.ones(n)
    out_norm = torch.pow(out_degs, -0.5) if agg == "sym" else torch.ones(n)
    return in_norm, out_norm


# ----------------------------------------------------------------------------- sigma
def act_fwd(z, act, slope=0.01):
    if act == "identity":
        return z
    if act == "relu":
        return torch.relu(z)
    if act == "leaky":
        return torch.nn.functional.leaky_relu(z, slope)
    if act == "gelu":
        return torch.nn.functional.gelu(z)
    if act == "gelu_tanh":
        return torch.nn.functional.gelu(z, approximate="tanh")
    raise ValueError(act)


def act_bwd(z, grad, act, slope=0.01):
    """d sigma(z) * grad, as torch's backward formulas compute it."""
    if act == "identity":
        return grad
    if act == "relu":
        return torch.where(z > 0, grad, torch.zeros_like(grad))
    if act == "leaky":
        return torch.where(z > 0, grad, grad * slope)
    if act in ("gelu", "gelu_tanh"):
        zz = z.detach().clone().requires_grad_(True)
        with torch.enable_grad():
            y = act_fwd(zz, act)
            (g,) = torch.autograd.grad(y, zz, grad)
        return g
    raise ValueError(act)


# ----------------------------------------------------------------------------- kernels
def _edge_coef(out_norm, in_norm, src, dst, agg):
    """``conv.py:45``: ``edges.src['out_norm'] * edges.dst['in_norm']`` (fp32 product first)."""
    if agg == "sym":
        return (out_norm[src] * in_norm[dst]).unsqueeze(-1)
    return None


def edge_agg_fwd(src, dst, num_nodes, Q, K, agg, act, slope=0.01):
    """S[v] = sum_{e:u->v} (n_out[u] n_in[v]) * sigma(Q[v] + K[u]); mean divides by deg.

    ``conv.py:43-45`` (message) + ``conv.py:63`` (update_all, fn.sum / fn.mean) restated.
    Accumulation is ``index_add`` in edge-id order == DGL CPU SpMM order per row.
    """
    src = torch.as_tensor(src, dtype=torch.int64)
    dst = torch.as_tensor(dst, dtype=torch.int64)
    in_deg = torch.bincount(dst, minlength=num_nodes)
    out_deg = torch.bincount(src, minlength=num_nodes)
    in_norm, out_norm = degree_norms(in_deg, out_deg, agg)
    z = Q.index_select(0, dst) + K.index_select(0, src)
    m = act_fwd(z, act, slope)
    c = _edge_coef(out_norm, in_norm, src, dst, agg)
    if c is not None:
        m = c * m
    S = torch.zeros((num_nodes, Q.shape[1]), dtype=m.dtype).index_add_(0, dst, m)
    if agg == "mean":
        S = S / in_deg.clamp(1, max(int(src.numel()), 1)).to(S.dtype).unsqueeze(-1)
    return S


def edge_agg_bwd(src, dst, num_nodes, Q, K, dS, agg, act, slope=0.01):
    """Analytic backward of ``edge_agg_fwd`` (autograd through ``conv.py:45,63``):
    t_e = (c_e) * g[v] with g = dS (mean: dS / deg), dz_e = sigma'(z_e) t_e,
    dQ[v] = sum over in-edges (edge order), dK[u] = sum over out-edges (edge order)."""
    src = torch.as_tensor(src, dtype=torch.int64)
    dst = torch.as_tensor(dst, dtype=torch.int64)
    in_deg = torch.bincount(dst, minlength=num_nodes)
    out_deg = torch.bincount(src, minlength=num_nodes)
    in_norm, out_norm = degree_norms(in_deg, out_deg, agg)
    g = dS
    if agg == "mean":
        g = dS / in_deg.clamp(1, max(int(src.numel()), 1)).to(dS.dtype).unsqueeze(-1)
    z = Q.index_select(0, dst) + K.index_select(0, src)
    t = g.index_select(0, dst)
    c = _edge_coef(out_norm, in_norm, src, dst, agg)
    if c is not None:
        t = t * c
    dz = act_bwd(z, t, act, slope)
    H = Q.shape[1]
    dQ = torch.zeros((num_nodes, H), dtype=dz.dtype).index_add_(0, dst, dz)
    dK = torch.zeros((num_nodes, H), dtype=dz.dtype).index_add_(0, src, dz)
    return dQ, dK


# ----------------------------------------------------------------------------- max
def max_first_wins(dst, num_nodes, M):
    """DGL ``fn.max`` over in-edges (``conv.py:41,63`` with agg_type='max'): elementwise max, the
    arg is the FIRST maximal edge in CSC order (= smallest edge id; DGL SpMMCmpCsr updates on
    strict >), rows without in-edges give 0 / arg -1.  Returns (Y, arg) with arg = edge ids."""
    dev = M.device                      # runs where M lives (CPU for the fixtures, GPU as a test checker)
    dst = torch.as_tensor(dst, dtype=torch.int64).to(dev)
    E, F = M.shape
    Y = torch.zeros((num_nodes, F), dtype=M.dtype, device=dev)
    arg = torch.full((num_nodes, F), -1, dtype=torch.int64, device=dev)
    if E == 0:
        return Y, arg
    idx = dst.unsqueeze(1).expand(E, F)
    Y = Y.scatter_reduce(0, idx, M, reduce="amax", include_self=False)
    eid = torch.arange(E, device=dev).unsqueeze(1).expand(E, F)
    cand = torch.where(M == Y[dst], eid, torch.full_like(eid, E))
    arg = torch.full((num_nodes, F), E, dtype=torch.int64, device=dev).scatter_reduce(0, idx, cand, reduce="amin")
    arg[arg == E] = -1
    return Y, arg


class _MaxFirstWins(torch.autograd.Function):
    @staticmethod
    def forward(ctx, M, dst, num_nodes):
        Y, arg = max_first_wins(dst, num_nodes, M)
        ctx.save_for_backward(arg, torch.as_tensor(dst, dtype=torch.int64))
        ctx.E = M.shape[0]
        return Y

    @staticmethod
    def backward(ctx, dY):
        arg, dst = ctx.saved_tensors
        E, F = ctx.E, dY.shape[1]
        dM = torch.zeros((E, F), dtype=dY.dtype, device=dY.device)
        hit = arg >= 0
        rows, cols = torch.nonzero(hit, as_tuple=True)
        dM[arg[rows, cols], cols] = dY[rows, cols]
        return dM, None, None


class _MaxGivenArg(_MaxFirstWins):
    """``fn.max`` evaluated on GIVEN arg edges (edge ids [V, F], -1 = empty row): Y[v, f] = M[arg, f],
    the gradient routed to that edge.  Used to score a result whose arg edges differ from this
    evaluation's own only on near-ties (the kernel's fp32 values rank two edges the other way):
    the oracle then follows the kernel's routing and everything else is compared as usual."""

    @staticmethod
    def forward(ctx, M, dst, num_nodes, arg):
        arg = torch.as_tensor(arg, dtype=torch.int64)
        hit = arg >= 0
        Y = torch.zeros((num_nodes, M.shape[1]), dtype=M.dtype)
        rows, cols = torch.nonzero(hit, as_tuple=True)
        Y[rows, cols] = M[arg[rows, cols], cols]
        ctx.save_for_backward(arg, torch.as_tensor(dst, dtype=torch.int64))
        ctx.E = M.shape[0]
        return Y

    @staticmethod
    def backward(ctx, dY):
        dM, _, _ = _MaxFirstWins.backward(ctx, dY)
        return dM, None, None, None


def max_tie_flips(M64, mag, dst, num_nodes, arg, c=16.0):
    """Check the arg edges ``arg`` ([V, F] edge ids) of an fp32 evaluation against the fp64 values
    M64 [E, F]: wherever ``arg`` is not the fp64 first arg-max ``a*``, the two edges must be a near-tie,
    |M64[a*] - M64[arg]| <= c * 2^-24 * max(mag[a*], mag[arg]) — within the fp32 rounding of values of
    magnitude ``mag`` (the sum of absolute terms that fed each M element).  Returns (n_flips, worst
    ratio gap / (2^-24 mag), n_violations)."""
    _, a64 = max_first_wins(dst, num_nodes, M64)
    arg = torch.as_tensor(arg, dtype=torch.int64)
    flip = (arg != a64)
    if not flip.any():
        return 0, 0.0, 0
    rows, cols = torch.nonzero(flip, as_tuple=True)
    ea, eb = a64[rows, cols], arg[rows, cols]
    assert bool((ea >= 0).all() and (eb >= 0).all()), "an empty row got an arg edge (or lost one)"
    gap = (M64[ea, cols] - M64[eb, cols]).abs()
    scale = torch.maximum(mag[ea, cols], mag[eb, cols]) * 2.0 ** -24
    ratio = gap / scale.clamp_min(1e-300)
    return int(flip.sum()), float(ratio.max()), int((ratio > c).sum())


def max_edge_values(src, dst, X, W_Q, b_Q, W_K, W_R, b_R, act, slope=0.01):
    """fp64 per-edge messages of the max form (conv.py:45-47: M = W_R sigma(Q[v] + K[u]) + b_R) and
    their magnitudes (the same expression over absolute values: |W_R| (|Q| + |K|) + |b_R|, with
    |Q| = |X| |W_Q|^T + |b_Q|), for :func:`max_tie_flips`."""
    src = torch.as_tensor(src, dtype=torch.int64)
    dst = torch.as_tensor(dst, dtype=torch.int64)
    X, W_Q, b_Q, W_K, W_R, b_R = (t.double() for t in (X, W_Q, b_Q, W_K, W_R, b_R))
    Q = X @ W_Q.t() + b_Q
    K = X @ W_K.t()
    fn = act if callable(act) else (lambda z: act_fwd(z, act, slope))
    A = fn(Q[dst] + K[src])
    M = A @ W_R.t() + b_R
    Qm = X.abs() @ W_Q.abs().t() + b_Q.abs()
    Km = X.abs() @ W_K.abs().t()
    mag = (Qm[dst] + Km[src]) @ W_R.abs().t() + b_R.abs()
    return M, mag


# ----------------------------------------------------------------------------- layer
def sigma_tie_flips(qk, src, dst, X, W_Q, b_Q, W_K, c=4.0):
    """sigma' near-ties: the elements z = Q[v] + K[u] whose sign differs between the kernel's own
    projection ``qk`` ([V, 2H] fp32, as the edge kernels saw it: fl(Q + K) has the sign of the exact
    sum) and an fp64 projection.  sigma' of the ReLU family jumps at 0, so ONE such element moves a
    gradient by a whole dA element (relL2 ~1e-3 at the test sizes): a result that flipped only where
    |z64| <= c * 2^-24 * (|X| |W_Q|^T + |b_Q| + |X| |W_K|^T) — i.e. inside the fp32 rounding of the
    projection — is scored against the fp64 oracle evaluated on ``qk`` (``reference_cpu_step(...,
    qk=qk)``).  Returns (n_flips, worst |z64| / (2^-24 mag), n_violations)."""
    src = torch.as_tensor(src, dtype=torch.int64)
    dst = torch.as_tensor(dst, dtype=torch.int64)
    X, W_Q, b_Q, W_K = (t.double() for t in (X, W_Q, b_Q, W_K))
    H = W_Q.shape[0]
    qk = torch.as_tensor(qk).double()
    z32 = qk[dst, :H] + qk[src, H:]
    z64 = (X @ W_Q.t() + b_Q)[dst] + (X @ W_K.t())[src]
    flip = (z32 > 0) != (z64 > 0)
    if not flip.any():
        return 0, 0.0, 0
    mag = (X.abs() @ W_Q.abs().t() + b_Q.abs())[dst] + (X.abs() @ W_K.abs().t())[src]
    ratio = z64[flip].abs() / (mag[flip] * 2.0 ** -24).clamp_min(1e-300)
    return int(flip.sum()), float(ratio.max()), int((ratio > c).sum())


def reference_cpu_step(src, dst, num_nodes, X, W_Q, b_Q, W_K, W_R, b_R, dY, agg, act,
                       slope=0.01, need_grads=True, max_arg=None, qk=None):
    """The reference's CPU dataflow for one SIRConv layer, fwd (+ autograd bwd).

    ``conv.py:49-67``: norms (51-57), K = X W_K^T, Q = X W_Q^T + b_Q (59-61),
    update_all(message_func, agg) (63) as DGL's edge-UDF path runs it (gathers, elementwise,
    index_add), Y = S W_R^T + b_R (65).  Returns Y and (if ``need_grads``) the gradients.
    ``max_arg`` (agg 'max' only): evaluate fn.max on these arg edges ([V, O] edge ids) instead of
    this evaluation's own first arg-max (:class:`_MaxGivenArg`).  ``qk`` ([V, 2H]): evaluate the
    layer on these projection VALUES (the gradients still flow through X W_Q^T + b_Q, X W_K^T) —
    the oracle conditioned on a kernel's own Q, K for :func:`sigma_tie_flips` near-ties.
    """
    src = torch.as_tensor(src, dtype=torch.int64)
    dst = torch.as_tensor(dst, dtype=torch.int64)
    params = [t.detach().clone().requires_grad_(need_grads) for t in (X, W_Q, b_Q, W_K, W_R, b_R)]
    X_, W_Q_, b_Q_, W_K_, W_R_, b_R_ = params
    with torch.set_grad_enabled(need_grads):
        K = torch.nn.functional.linear(X_, W_K_)
        Q = torch.nn.functional.linear(X_, W_Q_, b_Q_)
        if qk is not None:                  # values of qk, gradients through the projections
            qk = torch.as_tensor(qk).to(Q.dtype)
            H = Q.shape[1]
            Q = Q + (qk[:, :H] - Q).detach()
            K = K + (qk[:, H:] - K).detach()
        if callable(act) or agg == "max":
            # the general UDF dataflow (conv.py:43-47): sigma is any callable, max -> per-edge W_R
            fn = act if callable(act) else (lambda z: act_fwd(z, act, slope))
            a = fn(Q.index_select(0, dst) + K.index_select(0, src))
            if agg == "max" and max_arg is not None:
                Y = _MaxGivenArg.apply(torch.nn.functional.linear(a, W_R_, b_R_), dst, num_nodes, max_arg)
            elif agg == "max":
                Y = _MaxFirstWins.apply(torch.nn.functional.linear(a, W_R_, b_R_), dst, num_nodes)
            else:
                in_deg = torch.bincount(dst, minlength=num_nodes)
                out_deg = torch.bincount(src, minlength=num_nodes)
                in_norm, out_norm = degree_norms(in_deg, out_deg, agg)
                c = _edge_coef(out_norm, in_norm, src, dst, agg)
                m = c * a if c is not None else a
                S = torch.zeros((num_nodes, a.shape[1]), dtype=m.dtype).index_add(0, dst, m)
                if agg == "mean":
                    S = S / in_deg.clamp(1, max(int(src.numel()), 1)).to(S.dtype).unsqueeze(-1)
                Y = torch.nn.functional.linear(S, W_R_, b_R_)
        else:
            S = edge_agg_fwd(src, dst, num_nodes, Q, K, agg, act, slope)
            Y = torch.nn.functional.linear(S, W_R_, b_R_)
    out = {"Y": Y.detach()}
    if need_grads:
        Y.backward(dY)
        for name, p in zip(("dX", "dW_Q", "db_Q", "dW_K", "dW_R", "db_R"), params):
            out[name] = p.grad
    return out


def layer_fwd_bwd(src, dst, num_nodes, X, W_Q, b_Q, W_K, W_R, b_R, dY, agg, act, slope=0.01):
    """Whole-layer oracle with the analytic backward written out (no autograd), so each
    gradient formula is explicit."""
    src = torch.as_tensor(src, dtype=torch.int64)
    dst = torch.as_tensor(dst, dtype=torch.int64)
    Q = X @ W_Q.t() + b_Q
    K = X @ W_K.t()
    S = edge_agg_fwd(src, dst, num_nodes, Q, K, agg, act, slope)
    Y = S @ W_R.t() + b_R
    G = dY @ W_R                                     # dS (mean division inside edge_agg_bwd)
    dQ, dK = edge_agg_bwd(src, dst, num_nodes, Q, K, G, agg, act, slope)
    return {
        "Y": Y, "S": S, "Q": Q, "K": K, "dS": G, "dQ": dQ, "dK": dK,
        "dX": dQ @ W_Q + dK @ W_K, "dW_Q": dQ.t() @ X, "db_Q": dQ.sum(0),
        "dW_K": dK.t() @ X, "dW_R": dY.t() @ S, "db_R": dY.sum(0),
    }


def gelu_erf_scalar(x):
    """Scalar GELU(erf) used by small pure-Python checks."""
    return 0.5 * x * (1.0 + math.erf(x / math.sqrt(2.0)))

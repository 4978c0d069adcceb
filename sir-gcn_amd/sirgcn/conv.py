"""Drop-in ``SIRConv`` running its message passing on hand-written gfx950 kernels.

Mirrors briangodwinlim/SIR-GCN ``models/conv.py:7-67``:

* same constructor ``SIRConv(input_dim, hidden_dim, output_dim, activation, dropout=0,
  inner_bias=True, outer_bias=True, agg_type='sum')`` (``conv.py:32``) and attributes
  (``activation``, ``dropout``, ``linear_query``, ``linear_key`` (no bias, ``conv.py:37``),
  ``linear_relation``, ``_agg_type``) -> identical ``state_dict`` keys;
* same ``forward(graph, feat) -> Tensor[V, output_dim]`` (``conv.py:49``);
* same numerics: fp32 degree norms (``conv.py:51-57``), message
  ``(out_norm[u] * in_norm[v]) * sigma(eq[v] + ek[u])`` (``conv.py:45``), sum / mean (= sum /
  clamp(deg, 1)) / sym aggregation (``conv.py:41,63``), ``Y = W_R S + b_R`` (``conv.py:65``) so
  isolated destinations output ``b_R``.

What runs where: the two node projections are ONE GEMM against the concatenated [W_Q; W_K],
the edge aggregation and its backward are the edge kernels, W_R and every backward GEMM are the
split-fp16 MFMA GEMMs (``linalg``) — all HIP kernels of ``libsirconv.so`` (C ABI,
``include/sirconv.h``).  There is no CPU
path: a CPU tensor, a missing library or an unsupported sigma/agg raises.
"""
import torch
from torch import nn
import torch.nn.functional as F

from . import _native, linalg
from .graph import DEFAULT_CHUNK, get_plan


# Test instrumentation: when a list, every forward appends the [Q | K] the edge kernels read (detached
# copies, in call order), so a parity check can tell sigma' near-ties from errors (tests/test_stacks_gpu.py).
QK_TRACE = None


def _trace_qk(QK):
    if QK_TRACE is not None:
        QK_TRACE.append(QK.detach().clone())


def activation_code(act):
    """Map the reference's ``activation`` callable (``conv.py:32,45``) to a kernel code."""
    if isinstance(act, nn.LeakyReLU):
        return _native.ACT_LEAKY, float(act.negative_slope)
    if isinstance(act, nn.ReLU) or act in (torch.relu, F.relu):
        return _native.ACT_RELU, 0.0
    if isinstance(act, nn.GELU):
        return (_native.ACT_GELU_TANH if act.approximate == "tanh" else _native.ACT_GELU), 0.0
    if act is F.gelu:
        return _native.ACT_GELU, 0.0
    if isinstance(act, nn.Identity) or act is None:
        return _native.ACT_IDENTITY, 0.0
    if act is F.leaky_relu:
        return _native.ACT_LEAKY, 0.01
    raise NotImplementedError(
        f"SIRConv: activation {act!r} has no native kernel (supported: ReLU, LeakyReLU, GELU, Identity)")


def _storage_dtype(dtype, H):
    """Feature storage of the edge kernels for a QK of ``dtype``: the autocast dtypes run natively
    as 16-bit rows (fp32 math inside), everything else as fp32."""
    if dtype in (torch.bfloat16, torch.float16) and H % 4 == 0:
        return dtype
    return torch.float32


class EdgeAggregate(torch.autograd.Function):
    """S = update_all(message_func, agg) of ``conv.py:63`` on packed ``QK = [Q | K]`` ([V, 2H]).

    Under autocast (the reference's AMP path, ``heterophilous-datasets/train.py:75``) Q and K
    arrive as bf16/fp16: the kernels gather those 16-bit rows directly (half the bytes), compute
    z, sigma and the fp32 sum the reference's promoted messages get, and
    return S in the same 16-bit dtype — the cast ``linear_relation`` applies to the reference's
    fp32 S anyway.  The backward reads dS and writes dQ/dK in that dtype as well.

    Backward returns dQK written by the dst pass (dQ half) and the src pass (dK half).
    For sigma in {ReLU, LeakyReLU} (any H <= 1024; the sub-wave rows of H <= 128 write their record
    from the wave ballots, ``sir_mask_words``) the forward also stores the sign of every z = Q[v] + K[u] and the
    backward runs in sign-mask mode: no Q/K re-gather, QK not kept alive; results are bit-identical
    to the recompute mode."""

    use_mask = True
    dual = True          # one-launch backward (sir_edge_agg_bwd) where it applies

    @staticmethod
    def forward(ctx, QK, plan, H, agg, act, slope, grad_on=True):
        if QK.device.type != "cuda":
            raise RuntimeError("SIRConv native path needs a ROCm GPU tensor (no CPU fallback)")
        ctx.in_dtype = QK.dtype
        st = _storage_dtype(QK.dtype, H)
        QK = QK.contiguous().to(st)
        V = QK.shape[0]
        Q, K = QK[:, :H], QK[:, H:]
        in_norm, out_norm = plan.norms(agg)
        S = torch.empty((V, H), device=QK.device, dtype=st)
        partial = _partial(plan, H, QK.device)
        nw = _native.mask_words(H, act) if EdgeAggregate.use_mask else 0
        mask = None
        if nw and grad_on and QK.requires_grad:     # (inference: no mask; Function.forward runs under no_grad)
            mask = torch.empty((max(plan.dst.col.numel(), 1) * nw,), device=QK.device, dtype=torch.int64)
        _native.edge_agg_fwd(plan.dst, Q, K, in_norm, out_norm, agg, act, slope, S, partial, mask)
        if mask is not None:
            ctx.save_for_backward(mask)
        else:
            ctx.save_for_backward(QK)
        ctx.masked = mask is not None
        ctx.plan, ctx.H, ctx.agg, ctx.act, ctx.slope, ctx.V, ctx.st = plan, H, agg, act, slope, V, st
        return S

    @staticmethod
    def backward(ctx, dS):
        (saved,) = ctx.saved_tensors
        plan, H, agg, act, slope, V, st = ctx.plan, ctx.H, ctx.agg, ctx.act, ctx.slope, ctx.V, ctx.st
        G = dS.contiguous().to(st)
        dQK = torch.empty((V, 2 * H), device=G.device, dtype=st)
        if ctx.masked:
            Q = K = None
            mask = saved
        else:
            Q, K = saved[:, :H], saved[:, H:]
            mask = None
        edge_backward(plan, H, agg, act, slope, G, Q, K, mask, dQK)
        return dQK.to(ctx.in_dtype), None, None, None, None, None, None


def _partial(plan, H, device):
    n = max(plan.dst.n_slots, plan.src.n_slots)
    return torch.empty((max(n, 1) * H,), device=device, dtype=torch.float32) if n else None


def _slots(csr, H, device):
    return torch.empty((csr.n_slots * H,), device=device, dtype=torch.float32) if csr.n_slots else None


def edge_backward(plan, H, agg, act, slope, G, Q, K, mask, dQK, drop=None):
    """dQ -> dQK[:, :H], dK -> dQK[:, H:] (the backward of ``update_all``, conv.py:45,63).  Sign-mask
    mode runs both passes in one launch (``sir_edge_agg_bwd``; MEAN on G / deg formed first);
    recompute mode runs them one after the other (MEAN: the source pass reads the destination
    pass's G / deg).  ``drop``: the (seed, p) feature dropout of the forward's QK — the passes
    store dQK already multiplied by its mask and scale (the dropout's backward)."""
    in_norm, out_norm = plan.norms(agg)
    if mask is not None and EdgeAggregate.dual:
        if agg == "mean":
            # both passes of MEAN read g = G / deg(v) (the reference's DivBackward, rounded once to
            # the storage dtype): form it first, then the one-launch SUM backward on it is the MEAN
            # backward (bit-identical to the two-launch form, which divides inside the dQ pass)
            deg = plan.in_degree_f()
            G = torch.div(G, deg, out=torch.empty_like(G))  # fp32 math, one rounding to G's dtype, no fp32 temporary
            agg = "sum"
        _native.edge_agg_bwd(plan.dst, plan.src, G, mask, in_norm, out_norm, agg, act, slope, dQK[:, :H],
                             dQK[:, H:], _slots(plan.dst, H, G.device), _slots(plan.src, H, G.device), drop=drop)
        return
    partial = _partial(plan, H, G.device)
    Gm = torch.empty((G.shape[0], H), device=G.device, dtype=G.dtype) if agg == "mean" else None
    _native.edge_agg_bwd_dst(plan.dst, Q, K, G, in_norm, out_norm, agg, act, slope, dQK[:, :H], Gm, partial, mask,
                             drop=drop)
    _native.edge_agg_bwd_src(plan.src, K, Q, Gm if Gm is not None else G, out_norm, in_norm,
                             agg, act, slope, dQK[:, H:], partial, mask, drop=drop)


_tn = linalg.mm_tn


def _bias_grad(G):
    """sum over rows (native deterministic column sum when the layout allows)."""
    if (G.is_cuda and G.shape[1] % 4 == 0 and G.stride(1) == 1 and G.stride(0) % 4 == 0
            and G.data_ptr() % 16 == 0):
        return _native.col_sum(G)
    return G.sum(0)


def _weight_and_bias_grad(G, X, need_w, need_b):
    """nn.Linear autograd: dW = G^T X and db = sum_rows G.  When both are needed the column sums
    come out of the weight-gradient GEMM's own pass over G (``sir_gemm_tn`` colsum_a)."""
    if need_w and need_b:
        return _tn(G, X, colsum=True)
    if need_w:
        return _tn(G, X), None
    return None, (_bias_grad(G) if need_b else None)


def _weight_and_bias_grad16(G, X, need_w, need_b):
    """:func:`_weight_and_bias_grad` for the 16-bit tensors of the autocast layer: dW = G^T X and
    db = sum_rows G in fp32 (``sir_gemm_tn16``: exact 16-bit products, fp32 sums; no fp32 copies)."""
    if need_w:
        return linalg.mm_tn16(G, X, colsum=True) if need_b else (linalg.mm_tn16(G, X), None)
    return None, (_bias_grad(G.float()) if need_b else None)


class SIRConvFunction(torch.autograd.Function):
    """The whole layer (``conv.py:49-67``) with a hand-scheduled backward:

    forward : QK = X [W_Q; W_K]^T + [b_Q; 0]  (one GEMM)  ->  S = edge kernels  ->  Y = S W_R^T + b_R
    backward: G = dY W_R, dW_R = dY^T S (split-K), db_R = sum dY, dQ/dK = edge passes,
              dX = [dQ dK] [W_Q; W_K], [dW_Q; dW_K] = [dQ dK]^T X (split-K), db_Q = sum dQ.
    Feature dropout on Q and K (conv.py:60-61, training with p > 0): ``drop`` = (seed, p); the QK
    GEMM's epilogue applies the hashed mask and the backward edge passes apply the same mask to
    dQK (``sirconv_dropout.h``) — no mask tensor, no extra pass.  Used for fp32 inputs (the
    modular path covers the rest)."""

    @staticmethod
    def forward(ctx, X, W_Q, b_Q, W_K, W_R, b_R, plan, agg, act, slope, grad_on=True, drop=None):
        H = W_Q.shape[0]
        X = X.contiguous()
        # X [W_Q; W_K]^T + [b_Q; 0]: the small-batch kernel reads W_Q / W_K in place and biases the
        # Q half only (no cat / pad launches per step: small batches are launch-bound)
        QK = linalg.mm_wt_pair(X, W_Q, W_K, b_Q, drop=drop)
        _trace_qk(QK)
        V = QK.shape[0]
        in_norm, out_norm = plan.norms(agg)
        S = torch.empty((V, H), device=X.device, dtype=torch.float32)
        partial = _partial(plan, H, X.device)
        # needs_input_grad mirrors requires_grad even under torch.no_grad(): the caller passes the
        # grad mode, so inference forwards never write the per-edge sign mask
        training = grad_on and any(ctx.needs_input_grad[:6])
        nw = _native.mask_words(H, act) if (EdgeAggregate.use_mask and training) else 0
        mask = torch.empty((max(plan.dst.col.numel(), 1) * nw,), device=X.device, dtype=torch.int64) if nw else None
        _native.edge_agg_fwd(plan.dst, QK[:, :H], QK[:, H:], in_norm, out_norm, agg, act, slope, S, partial, mask)
        Y = linalg.mm_wt(S, W_R, b_R)
        ctx.save_for_backward(X, W_Q, W_K, W_R, S, mask if mask is not None else QK)
        ctx.masked = mask is not None
        ctx.plan, ctx.agg, ctx.act, ctx.slope, ctx.drop = plan, agg, act, slope, drop
        ctx.has_bq, ctx.has_br = b_Q is not None, b_R is not None
        return Y

    @staticmethod
    def backward(ctx, dY):
        X, W_Q, W_K, W_R, S, saved = ctx.saved_tensors
        plan, agg, act, slope = ctx.plan, ctx.agg, ctx.act, ctx.slope
        H = W_R.shape[1]
        V = X.shape[0]
        dY = dY.contiguous()
        G = linalg.mm_w(dY, W_R)
        dW_R, db_R = _weight_and_bias_grad(dY, S, ctx.needs_input_grad[4], ctx.has_br and ctx.needs_input_grad[5])
        if ctx.masked:
            Q = K = None
            mask = saved
        else:
            Q, K = saved[:, :H], saved[:, H:]
            mask = None
        dQK = torch.empty((V, 2 * H), device=X.device, dtype=torch.float32)
        edge_backward(plan, H, agg, act, slope, G, Q, K, mask, dQK, ctx.drop)
        dX = linalg.mm_w_pair(dQK, W_Q, W_K) if ctx.needs_input_grad[0] else None
        dW_Q = dW_K = db_Q = None
        need_bq = ctx.has_bq and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[3]:
            dW, cs = _weight_and_bias_grad(dQK, X, True, need_bq)     # cs: column sums of [dQ dK]
            dW_Q, dW_K = dW[:H], dW[H:]
            db_Q = cs[:H] if need_bq else None
        elif need_bq:
            db_Q = _bias_grad(dQK[:, :H])
        return dX, dW_Q, db_Q, dW_K, dW_R, db_R, None, None, None, None, None, None


class SIRConvFunction16(torch.autograd.Function):
    """The whole layer under autocast (bf16 / fp16 ``dt``, the reference's AMP path,
    ``heterophilous-datasets/train.py:75``), hand-scheduled like :class:`SIRConvFunction`:

    forward : QK = X [W_Q; W_K]^T + [b_Q; 0] in dt (autocast's nn.Linear; native 16-bit MFMA
              ``sir_gemm_nt16`` with the X.to(dt) cast fused into its loads)
              -> S = edge kernels on dt rows (fp32 math inside) -> Y = S W_R^T + b_R in dt
    backward: G = dY W_R in dt and dX = dQK [W_Q; W_K] (``sir_gemm_nt16``; dX for an fp32 X
              straight from the fp32 accumulator); the weight gradients dW = dY^T S, [dQ dK]^T X
              and the bias gradients — contractions over all V node rows — on the native 16-bit
              TN kernel (exact 16-bit products, fp32 sums), fp32 like the parameters.  Small
              graphs (and shapes the kernels do not take) run the same dataflow on torch's
              half-precision GEMMs (``linalg.mm16_*``)."""

    @staticmethod
    def forward(ctx, X, W_Q, b_Q, W_K, W_R, b_R, plan, agg, act, slope, grad_on, dt, drop=None):
        H = W_Q.shape[0]
        W_cat = torch.cat([W_Q, W_K], 0)
        b_cat = F.pad(b_Q, (0, H)) if b_Q is not None else None
        X = X.contiguous()
        if X.dtype == dt:
            Xh = X
            QK = linalg.mm16_wt(X, W_cat, b_cat, dt, drop=drop)
        else:       # X.to(dt) fused into the GEMM's loads; the rounded X (for dW) written by it
            Xh = torch.empty(X.shape, dtype=dt, device=X.device)
            QK = linalg.mm16_wt(X, W_cat, b_cat, dt, acopy=Xh, drop=drop)
        _trace_qk(QK)
        V = QK.shape[0]
        in_norm, out_norm = plan.norms(agg)
        S = torch.empty((V, H), device=X.device, dtype=dt)
        partial = _partial(plan, H, X.device)
        training = grad_on and any(ctx.needs_input_grad[:6])
        nw = _native.mask_words(H, act) if (EdgeAggregate.use_mask and training) else 0
        mask = torch.empty((max(plan.dst.col.numel(), 1) * nw,), device=X.device, dtype=torch.int64) if nw else None
        _native.edge_agg_fwd(plan.dst, QK[:, :H], QK[:, H:], in_norm, out_norm, agg, act, slope, S, partial, mask)
        Y = linalg.mm16_wt(S, W_R, b_R, dt)
        ctx.save_for_backward(Xh, W_cat, W_R, S, mask if mask is not None else QK)
        ctx.masked = mask is not None
        ctx.plan, ctx.agg, ctx.act, ctx.slope, ctx.x_dtype, ctx.dt, ctx.drop = plan, agg, act, slope, X.dtype, dt, drop
        ctx.has_bq, ctx.has_br = b_Q is not None, b_R is not None
        return Y

    @staticmethod
    def backward(ctx, dY):
        Xh, W_cat, W_R, S, saved = ctx.saved_tensors
        plan, agg, act, slope, dt = ctx.plan, ctx.agg, ctx.act, ctx.slope, ctx.dt
        H = W_R.shape[1]
        V = Xh.shape[0]
        dY = dY.contiguous().to(dt)
        G = linalg.mm16_w(dY, W_R, dt)
        dW_R = db_R = None
        if ctx.needs_input_grad[4] or ctx.needs_input_grad[5]:
            dW_R, db_R = _weight_and_bias_grad16(dY, S, ctx.needs_input_grad[4],
                                                 ctx.has_br and ctx.needs_input_grad[5])
        if ctx.masked:
            Q = K = None
            mask = saved
        else:
            Q, K = saved[:, :H], saved[:, H:]
            mask = None
        dQK = torch.empty((V, 2 * H), device=Xh.device, dtype=dt)
        edge_backward(plan, H, agg, act, slope, G, Q, K, mask, dQK, ctx.drop)
        # dX straight from the fp32 accumulator for an fp32 input (no 16-bit rounding, no cast pass)
        dX = linalg.mm16_w(dQK, W_cat, dt, out_dtype=ctx.x_dtype) if ctx.needs_input_grad[0] else None
        dW_Q = dW_K = db_Q = None
        need_bq = ctx.has_bq and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[3] or need_bq:
            dW, cs = _weight_and_bias_grad16(dQK, Xh, True, need_bq)
            dW_Q, dW_K = dW[:H], dW[H:]
            db_Q = cs[:H] if need_bq else None
        return dX, dW_Q, db_Q, dW_K, dW_R, db_R, None, None, None, None, None, None, None


class SIRConv(nn.Module):
    r"""Soft-Isomorphic Relational Graph Convolution (SIR-GCN), MI355X-native.

    .. math::  h_u^* = \sum_{v \in \mathcal{N}(u)} W_R \, \sigma(W_Q h_u + W_K h_v)

    Same parameters as the reference (``conv.py:13-31``).  ``sum``/``mean``/``sym`` with an
    elementwise sigma (ReLU, LeakyReLU, GELU, Identity) run on the fused edge kernels; ``max`` with
    an elementwise sigma and a ``Sequential(act, Linear, ReLU)`` sigma run on the fused edge-MLP
    kernels (``sirgcn.edgemlp``); any other sigma callable runs on the edge-materialised native
    path (``sirgcn.generic``).
    """

    use_fused = True      # whole-layer Function when dropout is off and inputs are fp32
    fuse_edge_mlp = True  # Sequential sigma / max aggregation on the fused edge-MLP kernels (sirgcn.edgemlp)
    native_linear = True  # projections of the non-fused routes on the native GEMMs (linalg.linear)

    def __init__(self, input_dim, hidden_dim, output_dim, activation, dropout=0, inner_bias=True,
                 outer_bias=True, agg_type='sum'):
        super().__init__()
        if agg_type not in ("sum", "mean", "sym", "max"):
            raise AttributeError(f"module 'dgl.function' has no attribute '{agg_type}'")
        self.activation = activation
        self.dropout = nn.Dropout(dropout)
        self.linear_query = nn.Linear(input_dim, hidden_dim, bias=inner_bias)
        self.linear_key = nn.Linear(input_dim, hidden_dim, bias=False)
        self.linear_relation = nn.Linear(hidden_dim, output_dim, bias=outer_bias)
        self._agg_type = agg_type
        self.chunk = DEFAULT_CHUNK
        # a one-element device seed handed in by a caller that drew the seeds of several layers in
        # one op (sirgcn.stacks.SIRStack), consumed by the next forward's _drop
        self.step_seed = None

    def _drop(self, device):
        """(seed, p) of this forward's fused feature dropout (conv.py:35,60-61), or None (eval / p = 0).
        The seed is a one-element int64 tensor drawn ON THE DEVICE from torch's CUDA generator — where
        the reference's nn.Dropout draws its bits — and read by the kernels from device memory: no
        host sync, the CPU RNG stream is untouched, and a forward captured in a HIP graph draws a
        fresh mask on every replay (the captured randint is graph-safe philox)."""
        if not (self.training and self.dropout.p > 0):
            self.step_seed = None
            return None
        seed, self.step_seed = self.step_seed, None
        if seed is None or seed.device != torch.device(device):
            seed = torch.randint(0, 2 ** 62, (1,), device=device, dtype=torch.int64)
        return seed, float(self.dropout.p)

    def _linear(self, x, W, b):
        """nn.Linear on the native GEMMs (``linalg.linear``; torch's F.linear when disabled or for
        operands the kernels do not take)."""
        if self.native_linear:
            return linalg.linear(x, W, b)
        return F.linear(x, W, b)

    def _relation(self, S):
        """``linear_relation`` (conv.py:65) — native when it is still the constructor's nn.Linear."""
        lin = self.linear_relation
        if type(lin) is nn.Linear:
            return self._linear(S, lin.weight, lin.bias)
        return lin(S)

    def _project(self, feat_key, feat_query):
        """K = drop(X W_K^T), Q = drop(X W_Q^T + b_Q) (``conv.py:60-61``) as ONE GEMM -> [V, 2H]."""
        H = self.linear_query.out_features
        if feat_key is feat_query:
            W = torch.cat([self.linear_query.weight, self.linear_key.weight], 0)
            b = None
            if self.linear_query.bias is not None:
                b = torch.cat([self.linear_query.bias, self.linear_query.bias.new_zeros(H)])
            QK = self._linear(feat_query, W, b)
        else:
            QK = torch.cat([self._linear(feat_query, self.linear_query.weight, self.linear_query.bias),
                            self._linear(feat_key, self.linear_key.weight, None)], 1)
        if self.training and self.dropout.p > 0:
            QK = self.dropout(QK)   # independent masks for Q and K, as two nn.Dropout calls
        _trace_qk(QK)
        return QK

    def forward(self, graph, feat):
        try:
            return self._forward(graph, feat)
        finally:
            self.step_seed = None          # a handed-in seed serves this one forward, whatever route ran

    def _forward(self, graph, feat):
        if isinstance(feat, tuple):          # expand_as_pair: (src feats, dst feats)
            feat_key, feat_query = feat
        else:
            feat_key = feat_query = feat
        if feat_query.dim() != 2:
            raise ValueError("SIRConv expects 2-D node features [V, input_dim]")
        if feat_query.device.type != "cuda":
            raise RuntimeError("SIRConv native path needs a ROCm GPU tensor (no CPU fallback)")
        plan = get_plan(graph, feat_query.device, self.chunk)
        if plan.num_nodes != feat_query.shape[0]:
            raise ValueError(f"feat has {feat_query.shape[0]} rows, graph has {plan.num_nodes} nodes")
        try:
            act, slope = activation_code(self.activation)
        except NotImplementedError:
            act = None
        H = self.linear_query.out_features
        if self.fuse_edge_mlp and feat_query.dtype != torch.float64:
            from .edgemlp import EdgeMaxLinear, EdgeMLPSum, max_supported, seq_sigma
            if self._agg_type == "max" and act is not None and \
                    max_supported(H, self.linear_relation.out_features):
                # conv.py:46-47 + fn.max: per-edge W_R fused with the gather and the running max
                QK = self._project(feat_key, feat_query)
                Y = EdgeMaxLinear.apply(QK, self.linear_relation.weight, self.linear_relation.bias, plan, H, act,
                                        slope)
                return Y.to(QK.dtype)
            sq = seq_sigma(self.activation, H) if act is None and self._agg_type != "max" else None
            if sq is not None:
                # conv.py:45 with sigma = Sequential(act1, Linear, act2): the Linear runs inside the edge loop
                a1, sl, lin, a2 = sq
                QK = self._project(feat_key, feat_query)
                S = EdgeMLPSum.apply(QK, lin.weight, lin.bias, plan, H, self._agg_type, a1, sl, a2)
                return self._relation(S.to(QK.dtype))
        if act is None or self._agg_type == "max":
            from .generic import generic_forward       # edge-materialised native path
            return generic_forward(self, plan, feat_key, feat_query)
        fused = (self.use_fused and feat_key is feat_query and feat_query.dtype == torch.float32 and feat_query.is_cuda
                 and not torch.is_autocast_enabled() and self.linear_query.weight.dtype == torch.float32)
        if fused:
            return self._fused(SIRConvFunction, feat_query, plan, act, slope)
        if (self.use_fused and feat_key is feat_query and torch.is_autocast_enabled()
                and feat_query.dtype in (torch.float32, torch.bfloat16, torch.float16)
                and self.linear_query.weight.dtype == torch.float32):
            dt = torch.get_autocast_dtype("cuda")
            if dt in (torch.bfloat16, torch.float16):
                with torch.autocast("cuda", enabled=False):
                    return self._fused(SIRConvFunction16, feat_query, plan, act, slope, dt)
        QK = self._project(feat_key, feat_query)
        S = EdgeAggregate.apply(QK, plan, H, self._agg_type, act, slope, torch.is_grad_enabled())
        return self._relation(S)

    def _fused(self, fn, X, plan, act, slope, *dt):
        """The whole-layer Function ``fn`` (SIRConvFunction / SIRConvFunction16).  Widths that are not
        multiples of 4 (the reference's own H = 75 / 95, zinc/train.py:206, ogbn-arxiv/train.py:303)
        run on zero-padded copies: the padded columns of Q, K are exactly 0, sigma(0) = 0 for every
        supported sigma and every gradient reaching them is 0, so the padded layer computes the same
        values; the pads' autograd slices the gradients back to the parameters' shapes."""
        W_Q, b_Q, W_K = self.linear_query.weight, self.linear_query.bias, self.linear_key.weight
        W_R, b_R = self.linear_relation.weight, self.linear_relation.bias
        (H, d), O = W_Q.shape, W_R.shape[0]
        Hp, dp, Op = -(-H // 4) * 4, -(-d // 4) * 4, -(-O // 4) * 4
        if (Hp, dp, Op) != (H, d, O):
            W_Q = F.pad(W_Q, (0, dp - d, 0, Hp - H))
            b_Q = F.pad(b_Q, (0, Hp - H)) if b_Q is not None else None
            W_K = F.pad(W_K, (0, dp - d, 0, Hp - H))
            W_R = F.pad(W_R, (0, Hp - H, 0, Op - O))
            b_R = F.pad(b_R, (0, Op - O)) if b_R is not None else None
            X = F.pad(X, (0, dp - d)) if dp != d else X
        Y = fn.apply(X, W_Q, b_Q, W_K, W_R, b_R, plan, self._agg_type, act, slope, torch.is_grad_enabled(), *dt,
                     self._drop(X.device))
        return Y[:, :O] if Op != O else Y

    def extra_repr(self):
        return f"agg_type={self._agg_type!r}"

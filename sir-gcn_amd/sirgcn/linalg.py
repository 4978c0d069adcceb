"""The layer's projection GEMMs on the native split-fp16 MFMA kernels (``sir_gemm_nt`` /
``sir_gemm_tn``, include/sirconv.h).

These are the nn.Linear calls of the reference (``conv.py:60-61`` Q/K, ``conv.py:65`` W_R) and
their autograd: ``mm_wt`` = A W^T (+ b) (forward projections), ``mm_w`` = A W (G = dY W_R,
dX = dQK [W_Q; W_K]), ``mm_tn`` = A^T B (the weight gradients, contraction over the node rows).
fp32 in / fp32 out at fp32 accuracy (tests/test_gemm_gpu.py).  Operands the kernels do not take
(CPU tensors of the gloo rehearsals, non-fp32, feature widths not a multiple of 4, unaligned
views, fewer than ``MIN_ROWS`` node rows) go to torch's own GEMM; ``USE_NATIVE = False`` forces that
for A/B runs.
"""
import os

import torch

from . import _native

USE_NATIVE = True
MAX_DIM = 65536          # N, K (and M, N of the TN GEMM) limit of the native kernels
MAX_LD = 1 << 20         # SIR_GEMM_MAX_LD (include/sirconv.h)
# Fewest node rows for the native route.  0: every batch size runs native — below 16,384 rows the
# library itself switches to its one-wave-per-tile kernels (k_gemm_nt_s / k_gemm_tn_s, bit-identical
# to the block-tiled NT kernels) that fill the chip at config 5's 1.6k-node and config 1's 5k-node
# batches (profiles/r03_ab_gemm_small.txt).  A positive value sends smaller batches to torch's fp32
# GEMM (hipBLASLt) instead.
DEFAULT_MIN_ROWS = 0
MIN_ROWS = int(os.environ.get("SIRGCN_GEMM_MIN_ROWS", DEFAULT_MIN_ROWS))


def _ok(t):
    return (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1 and t.shape[0] >= MIN_ROWS
            and t.stride(0) % 4 == 0 and t.shape[1] % 4 == 0 and t.data_ptr() % 16 == 0
            and t.shape[1] <= MAX_DIM and t.stride(0) <= MAX_LD)


def _w_ok(W, n_out):
    return W.is_cuda and W.dtype == torch.float32 and n_out % 4 == 0 and n_out <= MAX_DIM


# Below this many rows the weight is read as fp32 by the GEMM itself (sir_gemm_nt_direct: the
# LDS-tiled k_gemm_lt, 64 x 32 tiles, both operands split in the kernel) instead of being packed
# first: at config 5's 1.6k rows the packing pass cost as much as the product
# (profiles/r03_ab_gemm_small.txt, profiles/r05_small_gemm.txt).
DIRECT_ROWS = int(os.environ.get("SIRGCN_GEMM_DIRECT_ROWS", 8192))


def _direct_ok(A, W):
    return (A.shape[0] < DIRECT_ROWS and W.stride(1) == 1 and W.stride(0) <= MAX_LD and W.data_ptr() % 4 == 0)


def mm_wt(A, W, bias=None, out=None, drop=None):
    """A W^T + bias (nn.Linear); W [N, K].  ``drop``: (seed, p) feature dropout of the result
    (the QK projection, conv.py:60-61), applied in the native GEMM's epilogue — or, on the torch
    path, by ``sir_dropout_apply`` with the same hashed mask."""
    if (USE_NATIVE and _ok(A) and _w_ok(W, W.shape[0])
            and (bias is None or (bias.is_contiguous() and bias.data_ptr() % 16 == 0))
            and (out is None or _ok(out))):
        if _direct_ok(A, W):
            return _native.gemm_nt_direct(A, W, False, bias, out, drop=drop)
        return _native.gemm_nt(A, _native.gemm_pack(W.contiguous()), bias, out, drop=drop)
    if out is None:
        out = torch.addmm(bias, A, W.t()) if bias is not None else torch.mm(A, W.t())
    elif bias is not None:
        torch.addmm(bias, A, W.t(), out=out)
    else:
        torch.mm(A, W.t(), out=out)
    if drop is not None:
        _native.dropout_apply(out, drop)
    return out


def mm_w(A, W, out=None):
    """A W; W [K, N] (into ``out`` when given)."""
    if USE_NATIVE and _ok(A) and _w_ok(W, W.shape[1]) and (out is None or _ok(out)):
        if _direct_ok(A, W):
            return _native.gemm_nt_direct(A, W, True, out=out)
        return _native.gemm_nt(A, _native.gemm_pack(W.contiguous(), trans=True), out=out)
    if out is None:
        return torch.mm(A, W)
    return torch.mm(A, W, out=out)


def _lt_nt_env():
    """``SIR_LT_NT`` as the library reads it (atoi; unset / empty: -1 = by shape)."""
    e = os.environ.get("SIR_LT_NT", "")
    if not e:
        return -1
    digits = e.strip()
    n = len(digits) - len(digits.lstrip("+-"))
    while n < len(digits) and digits[n].isdigit():
        n += 1
    try:
        return int(digits[:n])
    except ValueError:
        return 0


def _pair_ok(A, W, W2, trans):
    """The two-part weight (``sir_gemm_nt_direct2``) runs only on the LDS-tiled kernel: the same
    conditions as run_gemm_nt_direct's route to it (SIR_LT_NT != 0, every byte offset of a tile's
    resource in 29 bits), else the caller takes the cat + pad route."""
    K = A.shape[1]
    return (USE_NATIVE and _ok(A) and A.shape[0] < DIRECT_ROWS and _lt_nt_env() != 0
            and 128 * A.stride(0) < (1 << 29)
            and all(w.is_cuda and w.dtype == torch.float32 and w.dim() == 2 and w.stride(1) == 1
                    and w.stride(0) % 4 == 0 and w.stride(0) <= MAX_LD and w.data_ptr() % 16 == 0
                    and (K * w.stride(0) if trans else 128 * w.stride(0)) < (1 << 29) for w in (W, W2)))


def mm_wt_pair(A, W, W2, bias=None, drop=None):
    """A [W; W2]^T + [bias; 0] (the layer's QK = X [W_Q; W_K]^T + [b_Q; 0], conv.py:60-61): on the
    small-batch route the kernel reads W and W2 where they lie and adds the bias to the first
    W.shape[0] outputs only (``sir_gemm_nt_direct2``) — no concatenated weight, no padded bias per
    step; elsewhere the cat + pad + :func:`mm_wt`."""
    n1 = W.shape[0]
    if (_pair_ok(A, W, W2, False) and n1 % 4 == 0 and W2.shape[0] % 4 == 0
            and (bias is None or (bias.is_cuda and bias.dtype == torch.float32 and bias.is_contiguous()
                                  and bias.data_ptr() % 16 == 0))):
        return _native.gemm_nt_direct2(A, W, W2, False, bias, n1 if bias is not None else 0, drop=drop)
    Wc = torch.cat([W, W2], 0)
    return mm_wt(A, Wc, torch.nn.functional.pad(bias, (0, W2.shape[0])) if bias is not None else None, drop=drop)


def mm_w_pair(A, W, W2):
    """A [W; W2] (the layer's dX = [dQ dK] [W_Q; W_K]): in place on the small-batch route, else the
    cat + :func:`mm_w`."""
    if _pair_ok(A, W, W2, True) and W.shape[1] % 4 == 0:
        return _native.gemm_nt_direct2(A, W, W2, True)
    return mm_w(A, torch.cat([W, W2], 0))


def mm_w_dact(A, W, gate, act, slope, gate_mask=None):
    """sigma'(gate) * (A W) for the ReLU family (W [K, N]; ``gate`` the activation's input or output,
    same sign; ``gate_mask``: its sign words, N = 256): native with the activation backward in the
    GEMM epilogue when the operands allow, else torch's mm + threshold / leaky_relu backward."""
    if (USE_NATIVE and _ok(A) and _w_ok(W, W.shape[1]) and _ok(gate) and gate.shape == (A.shape[0], W.shape[1])
            and gate.stride(0) == W.shape[1]):
        mask = gate_mask if W.shape[1] == 256 else None
        return _native.gemm_nt_dact(A, _native.gemm_pack(W.contiguous(), trans=True), gate, act, slope, gate_mask=mask)
    g = torch.mm(A, W)
    if act == _native.ACT_RELU:
        return torch.ops.aten.threshold_backward(g, gate, 0.0)
    return torch.ops.aten.leaky_relu_backward(g, gate, slope, False)


def _tn_ok(t):
    return (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1 and t.shape[0] >= MIN_ROWS
            and 0 < t.shape[1] <= MAX_DIM and t.stride(0) <= MAX_LD)


def mm_tn(A, B, colsum=False):
    """A^T B for tall A [R, M], B [R, N] (the weight gradients); with ``colsum`` also A.sum(0)
    (the bias gradient of the same linear), from the same pass: returns (A^T B, colsum)."""
    if USE_NATIVE and _tn_ok(A) and _tn_ok(B):
        return _native.gemm_tn(A, B, colsum=colsum)
    out = _tn_torch(A, B)
    return (out, A.sum(0)) if colsum else out


def _tn16_ok(t):
    return (t.is_cuda and t.dtype in (torch.bfloat16, torch.float16) and t.dim() == 2 and t.stride(1) == 1
            and t.shape[0] >= MIN_ROWS_16 and 0 < t.shape[1] <= MAX_DIM and t.shape[1] % 2 == 0
            and t.stride(0) % 2 == 0 and t.stride(0) <= MAX_LD and t.data_ptr() % 4 == 0)


# The 16-bit TN kernel moves half the bytes and does a third of the MFMA work of the split one;
# it still splits the rows over >= 2048-row ranges, so below this it cannot fill the chip.
DEFAULT_MIN_ROWS_16 = 16384
MIN_ROWS_16 = DEFAULT_MIN_ROWS_16


def mm_tn16(A, B, colsum=False):
    """A^T B (and A.sum(0) with ``colsum``) in fp32 for bf16 / fp16 A [R, M], B [R, N]: the weight
    and bias gradients of a half-precision nn.Linear (autocast), with fp32 accumulation of the
    exact 16-bit products.  Native ``sir_gemm_tn16`` when the operands allow, else torch on the
    values widened to fp32 (the same products, summed in fp32)."""
    if USE_NATIVE and A.dtype == B.dtype and _tn16_ok(A) and _tn16_ok(B):
        return _native.gemm_tn16(A, B, colsum=colsum)
    return mm_tn(A.float(), B.float(), colsum=colsum)


class _Linear(torch.autograd.Function):
    """nn.Linear (``y = x W^T + b``) with forward and backward on the native GEMMs: y = mm_wt,
    dx = mm_w(dy, W), (dW, db) = mm_tn(dy, x, colsum) — the weight and bias gradients from one pass."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return mm_wt(x, W, b)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dy = dy.contiguous()
        dx = mm_w(dy, W) if ctx.needs_input_grad[0] else None
        dW = db = None
        need_b = ctx.has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            if need_b:
                dW, db = mm_tn(dy, x, colsum=True)
            else:
                dW = mm_tn(dy, x)
        elif need_b:
            db = dy.sum(0)
        return dx, dW, db


class _Linear16(torch.autograd.Function):
    """Autocast's nn.Linear (``F.linear(x.to(dt), W.to(dt), b.to(dt))``) on the native 16-bit
    kernels: y = mm16_wt (x.to(dt) fused into the loads, the rounded x written for dW only when W
    needs a gradient), dx = mm16_w(dy, W) in x's dtype straight from the fp32 accumulator, and
    (dW, db) = mm_tn16(dy, x) in fp32 like the parameters (exact 16-bit products, fp32 sums)."""

    @staticmethod
    def forward(ctx, x, W, b, dt):
        xh = x
        if x.dtype != dt and ctx.needs_input_grad[1]:
            xh = torch.empty(x.shape, dtype=dt, device=x.device)
            y = mm16_wt(x, W, b, dt, acopy=xh)
        else:
            y = mm16_wt(x, W, b, dt)
        ctx.save_for_backward(xh if ctx.needs_input_grad[1] else None, W)
        ctx.has_b, ctx.x_dtype, ctx.dt = b is not None, x.dtype, dt
        return y

    @staticmethod
    def backward(ctx, dy):
        xh, W = ctx.saved_tensors
        dt = ctx.dt
        dy = dy.contiguous().to(dt)
        dx = mm16_w(dy, W, dt, out_dtype=ctx.x_dtype) if ctx.needs_input_grad[0] else None
        dW = db = None
        need_b = ctx.has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            dW, db = mm_tn16(dy, xh, colsum=True) if need_b else (mm_tn16(dy, xh), None)
        elif need_b:
            db = dy.float().sum(0)
        return dx, dW, db, None


def linear(x, W, b=None):
    """``F.linear(x, W, b)`` (the reference's ``nn.Linear`` calls, conv.py:60-61,65) on the native
    split-fp16 GEMMs for fp32 GPU operands the kernels take; under a bf16 / fp16 autocast (the
    reference's AMP path, heterophilous-datasets/train.py:75) on the native 16-bit GEMMs
    (:class:`_Linear16`) for shapes those take; anything else (fp64, other layouts, CPU tensors,
    small or odd-shaped autocast operands) is torch's own ``F.linear``."""
    if (USE_NATIVE and torch.is_autocast_enabled() and x.dim() == 2 and W.dim() == 2 and x.is_cuda
            and W.dtype == torch.float32 and W.is_cuda and (b is None or (b.dtype == torch.float32 and b.is_cuda))):
        dt = torch.get_autocast_dtype("cuda")
        xc = x if x.stride(1) == 1 else x.contiguous()
        if dt in (torch.bfloat16, torch.float16) and _nt16_ok(xc, W.shape[1], W.shape[0], dt):
            with torch.autocast("cuda", enabled=False):
                return _Linear16.apply(xc, W, b, dt)
        return torch.nn.functional.linear(x, W, b)
    if (USE_NATIVE and not torch.is_autocast_enabled() and x.dim() == 2 and W.dim() == 2
            and x.dtype == torch.float32 and W.dtype == torch.float32 and (b is None or b.dtype == torch.float32)):
        xc = x if x.stride(1) == 1 else x.contiguous()
        if _ok(xc) and _w_ok(W, W.shape[0]) and W.shape[1] % 4 == 0 and W.is_contiguous() \
                and (b is None or b.is_cuda):
            return _Linear.apply(xc, W, b.contiguous() if b is not None else None)
    return torch.nn.functional.linear(x, W, b)


def _tn_torch(A, B):
    """torch A^T B; long-K shapes run as k row blocks of one batched GEMM (hipBLASLt is 2x faster
    that way than as one GEMM) summed in a fixed order."""
    V = A.shape[0]
    k = 32
    while k > 1 and V // k < 4096:
        k //= 2
    if k == 1:
        return A.t() @ B
    n = (V // k) * k
    out = torch.bmm(A[:n].view(k, n // k, A.shape[1]).transpose(1, 2), B[:n].view(k, n // k, B.shape[1])).sum(0)
    if n < V:
        out += A[n:].t() @ B[n:]
    return out


# ---------------------------------------------------------------------------- 16-bit NT (autocast)
# The half-precision nn.Linear of the autocast path (forward x W^T + b, input gradient dY W) on the
# native 16-bit MFMA kernel (``sir_gemm_nt16``): fp32 A is rounded to the 16-bit type on load (the
# X.to(dt) cast fused in), the result is rounded once from the fp32 accumulator (or kept in fp32
# for the fp32 input's gradient).  Below MIN_ROWS_16 rows, or for shapes the kernel does not take,
# the same dataflow runs on torch's half-precision GEMM.
NT16_K = (128, 256, 512)


def _nt16_ok(A, K, N, dt, out=None):
    if out is not None and not (out.stride(1) == 1 and out.stride(0) % 8 == 0 and out.data_ptr() % 16 == 0):
        return False
    return (USE_NATIVE and A.is_cuda and A.dim() == 2 and A.stride(1) == 1 and A.dtype in (dt, torch.float32)
            and A.shape[0] >= MIN_ROWS_16 and K in NT16_K and N <= 512 and N % 8 == 0
            and A.stride(0) % (4 if A.dtype == torch.float32 else 8) == 0 and A.stride(0) <= MAX_LD
            and A.data_ptr() % 16 == 0)


def mm16_wt(A, W, bias, dt, out_dtype=None, acopy=None, drop=None, out=None):
    """F.linear(A.to(dt), W.to(dt), bias.to(dt)) (autocast's nn.Linear), result in ``out_dtype``
    (default dt).  ``acopy``: a [M, K] dt tensor that receives A.to(dt) when A is fp32.  ``drop``:
    (seed, p) feature dropout of the result (see ``mm_wt``)."""
    N, K = W.shape
    od = out_dtype or dt
    if _nt16_ok(A, K, N, dt, out) and (acopy is None or (A.dtype == torch.float32 and acopy.stride(1) == 1
                                                     and acopy.data_ptr() % 16 == 0)):
        b = bias.to(dt).float().contiguous() if bias is not None else None
        return _native.gemm_nt16(A, _native.gemm_pack16(W.contiguous().float(), dt), b, od, acopy, drop=drop,
                                 out=out)
    Ah = A.to(dt)
    if acopy is not None:
        acopy.copy_(Ah)
    res = torch.nn.functional.linear(Ah, W.to(dt), bias.to(dt) if bias is not None else None)
    res = res if res.dtype == od else res.to(od)
    if drop is not None:
        _native.dropout_apply(res, drop)
    if out is not None:
        out.copy_(res)
        return out
    return res


def mm16_w(A, W, dt, out_dtype=None):
    """(A.to(dt) @ W.to(dt)) in ``out_dtype`` (default dt): the input gradient of autocast's
    nn.Linear; W [K, N]."""
    K, N = W.shape
    od = out_dtype or dt
    if _nt16_ok(A, K, N, dt):
        return _native.gemm_nt16(A, _native.gemm_pack16(W.contiguous().float(), dt, trans=True), None, od)
    out = A.to(dt) @ W.to(dt)
    return out if out.dtype == od else out.to(od)

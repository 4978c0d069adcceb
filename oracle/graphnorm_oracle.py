"""CPU restatement of the reference GraphNorm (TEST INFRASTRUCTURE ONLY).

Reference: ``models/norm.py:7-29`` (briangodwinlim/SIR-GCN).  Per graph b of a batched graph
(nodes contiguous, ``batch_num_nodes``), per feature column:
    mean = sum_i x_i / n                       (norm.py:19-21; scatter_add in node order)
    d_i  = x_i - mean * mean_scale             (norm.py:22-23)
    std  = sqrt(sum_i d_i^2 / n + eps)         (norm.py:25-28)
    y_i  = weight * d_i / std + bias           (norm.py:29)
The variance is taken of the mean_scale-shifted values, as the reference does.

``ieee_sqrt=True`` takes the std through a correctly rounded square root (numpy).  The
reference's CPU ``torch.sqrt`` is vectorised (SLEEF/MKL) and is NOT correctly rounded for
wide tensors (about 0.7% of fp32 inputs differ by 1 ulp on this image), so the fixture's
``Y`` is bit-reproducible only with that same CPU kernel; a device sqrtf matches the IEEE
variant bit-for-bit instead.
"""
import numpy as np
import torch


def graph_norm_fwd(X, batch_num_nodes, weight, bias=None, mean_scale=None, eps=1e-5, ieee_sqrt=False):
    n = torch.as_tensor(batch_num_nodes, dtype=torch.int64)
    B = n.numel()
    gid = torch.repeat_interleave(torch.arange(B), n)
    F = X.shape[1]
    s = torch.zeros((B, F), dtype=X.dtype).index_add_(0, gid, X)
    mean = s / n.to(X.dtype).unsqueeze(1)
    ms = mean_scale if mean_scale is not None else 1
    d = X - mean[gid] * ms
    var = torch.zeros((B, F), dtype=X.dtype).index_add_(0, gid, d * d)
    pre = var / n.to(X.dtype).unsqueeze(1) + eps
    std = torch.from_numpy(np.sqrt(pre.numpy())) if ieee_sqrt else torch.sqrt(pre)
    Y = weight * d / std[gid]
    if bias is not None:
        Y = Y + bias
    return Y, mean, std


def graph_norm_bwd(X, dY, batch_num_nodes, weight, mean_scale, mean, std):
    """Analytic backward: A = sum gy*d, gd = w*gy/s - w*d*A/(n s^3),
    B = sum gd, dx = gd - ms*B/n; dw = sum gy*d/s, dms = -sum_b mean*B, db = sum gy."""
    n = torch.as_tensor(batch_num_nodes, dtype=torch.int64)
    B_ = n.numel()
    gid = torch.repeat_interleave(torch.arange(B_), n)
    nf = n.to(X.dtype).unsqueeze(1)
    ms = mean_scale if mean_scale is not None else torch.ones(X.shape[1], dtype=X.dtype)
    d = X - mean[gid] * ms
    s = std[gid]
    A = torch.zeros_like(mean).index_add_(0, gid, dY * d)
    gd = weight * dY / s - weight * d * A[gid] / (nf[gid] * s ** 3)
    Bsum = torch.zeros_like(mean).index_add_(0, gid, gd)
    dX = gd - ms * Bsum[gid] / nf[gid]
    dw = (A / std).sum(0)
    dms = (-(mean * Bsum)).sum(0)
    db = dY.sum(0)
    return dX, dw, db, dms

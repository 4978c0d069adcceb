"""CPU restatement of the reference SIREConv (TEST INFRASTRUCTURE ONLY).

Reference: ``models/conv.py:70-134`` (briangodwinlim/SIR-GCN).  Same dataflow as SIRConv with
an edge-feature term inside sigma, in the reference's operand order (``conv.py:108``):

    e   = efeat W_E^T                                   (conv.py:129, linear_edge, no bias)
    z_e = (Q[v] + K[u]) + e_uv                          (conv.py:108 / 110)
    m_e = (n_out[u] * n_in[v]) * sigma(z_e)             sum / mean / sym
    m_e = W_R sigma(z_e) + b_R                          max (first arg-max wins, DGL)
    Y   = W_R (sum_e m_e [/ deg]) + b_R                 sum / mean / sym
"""
import torch

from .sirconv_oracle import _MaxFirstWins, _edge_coef, act_fwd, degree_norms


def sire_reference_step(src, dst, num_nodes, X, efeat, W_Q, b_Q, W_K, W_E, W_R, b_R, dY, agg, act,
                        slope=0.01, need_grads=True):
    """One SIREConv layer fwd (+ autograd bwd) as DGL's edge-UDF path runs it; returns Y and the
    gradients dX, defeat, dW_Q, db_Q, dW_K, dW_E, dW_R, db_R."""
    src = torch.as_tensor(src, dtype=torch.int64)
    dst = torch.as_tensor(dst, dtype=torch.int64)
    params = [t.detach().clone().requires_grad_(need_grads) for t in (X, efeat, W_Q, b_Q, W_K, W_E, W_R, b_R)]
    X_, Ef_, W_Q_, b_Q_, W_K_, W_E_, W_R_, b_R_ = params
    F = torch.nn.functional
    with torch.set_grad_enabled(need_grads):
        K = F.linear(X_, W_K_)
        Q = F.linear(X_, W_Q_, b_Q_)
        Ee = F.linear(Ef_, W_E_)
        fn = act if callable(act) else (lambda z: act_fwd(z, act, slope))
        a = fn(Q.index_select(0, dst) + K.index_select(0, src) + Ee)
        if agg == "max":
            Y = _MaxFirstWins.apply(F.linear(a, W_R_, b_R_), dst, num_nodes)
        else:
            in_deg = torch.bincount(dst, minlength=num_nodes)
            out_deg = torch.bincount(src, minlength=num_nodes)
            in_norm, out_norm = degree_norms(in_deg, out_deg, agg)
            c = _edge_coef(out_norm, in_norm, src, dst, agg)
            m = c * a if c is not None else a
            S = torch.zeros((num_nodes, a.shape[1]), dtype=m.dtype).index_add(0, dst, m)
            if agg == "mean":
                S = S / in_deg.clamp(1, max(int(src.numel()), 1)).to(S.dtype).unsqueeze(-1)
            Y = F.linear(S, W_R_, b_R_)
    out = {"Y": Y.detach()}
    if need_grads:
        Y.backward(dY)
        for name, p in zip(("dX", "defeat", "dW_Q", "db_Q", "dW_K", "dW_E", "dW_R", "db_R"), params):
            out[name] = p.grad
    return out

"""BASELINE config 4 at its real size on one GPU: the S2 power-law graph (V = 2M, E = 40M),
H = d = O = 256, LeakyReLU(0.2), the whole layer through ``SIRConvFunction`` (the bench.py step).

* two runs are bit-identical (atomics-free kernels, fixed split-row combine order);
* the sign-mask backward equals the recompute backward bit for bit;
* the edge aggregation (S, dQ, dK) and the whole layer (Y, dX, every weight / bias gradient) are
  scored against a chunked torch evaluation of the reference dataflow in fp64 (truth) and fp32 (the
  reference's own rounding), per tensor as ``assert_parity`` does: relL2 vs fp64 <= max(1e-5,
  2 x the fp32 reference's).  The references run on the layer's own projection VALUES (captured
  through ``sirgcn.conv.QK_TRACE``; the QK GEMM itself is scored against the fp64 projection first),
  so sigma' near-ties of z = Q[v] + K[u] fall on the same side in every evaluation (tests/
  test_edgemlp_gpu.py: one flipped sign moves a gradient by ~1e-3 at these sizes).

The edge-cut of the same graph over 8 ranks (threaded, one GPU) is in tests/test_dist_gpu.py."""
import pytest
import torch
from torch import nn

from conftest import rel_err

from sirgcn import SIRConv, _native
import sirgcn.conv as sconv
from sirgcn.conv import EdgeAggregate
from sirgcn.graph import get_plan
from sirgcn.synth import NAMED, powerlaw_graph

pytestmark = pytest.mark.gpu
DEV = "cuda"
H = 256


@pytest.fixture(scope="module")
def s2():
    assert torch.cuda.is_available(), "GPU tests need the MI355X box"
    _native.load()
    V, E, a = NAMED["S2"]
    g = powerlaw_graph(V, E, a, seed=0)
    gen = torch.Generator(device=DEV).manual_seed(3)
    X = torch.randn(V, H, device=DEV, generator=gen)
    dY = torch.randn(V, H, device=DEV, generator=gen)
    return g, X, dY


def _layer(g, X, dY, agg, use_mask=True):
    torch.manual_seed(4)
    m = SIRConv(H, H, H, nn.LeakyReLU(0.2), 0, agg_type=agg).to(DEV)
    trace = []
    sconv.QK_TRACE = trace
    EdgeAggregate.use_mask = use_mask
    try:
        x = X.clone().requires_grad_(True)
        Y = m(g, x)
        Y.backward(dY)
    finally:
        sconv.QK_TRACE = None
        EdgeAggregate.use_mask = True
    torch.cuda.synchronize()
    out = {"Y": Y.detach(), "dX": x.grad, "dW_Q": m.linear_query.weight.grad, "db_Q": m.linear_query.bias.grad,
           "dW_K": m.linear_key.weight.grad, "dW_R": m.linear_relation.weight.grad,
           "db_R": m.linear_relation.bias.grad}
    return m, trace[0], out


def _edge_reference(src, dst, V, Q, K, G, agg, slope=0.2, step=1 << 20):
    """S, dQ, dK of the reference dataflow (conv.py:45,63 + autograd) in Q's dtype, edge-chunked."""
    in_deg = torch.bincount(dst, minlength=V)
    out_deg = torch.bincount(src, minlength=V)
    in_norm = torch.pow(in_deg.float().clamp(min=1), -0.5)
    out_norm = torch.pow(out_deg.float().clamp(min=1), -0.5)
    S = torch.zeros_like(Q)
    dQ = torch.zeros_like(Q)
    dK = torch.zeros_like(Q)
    for s in range(0, src.numel(), step):
        u, v = src[s:s + step], dst[s:s + step]
        z = Q[v] + K[u]
        m = torch.nn.functional.leaky_relu(z, slope)
        t = G[v]
        if agg == "sym":
            c = (out_norm[u] * in_norm[v]).unsqueeze(1).to(Q.dtype)
            m, t = c * m, t * c
        S.index_add_(0, v, m)
        dz = torch.where(z > 0, t, t * slope)
        dQ.index_add_(0, v, dz)
        dK.index_add_(0, u, dz)
        del z, m, t, dz
    return S, dQ, dK


def _layer_reference(src, dst, V, X, QK, m, dY, agg, dtype):
    """The whole layer on the projection values QK (gradients through the projections' formulas)."""
    W_Q, b_Q, W_K, W_R, b_R = (t.detach().to(dtype) for t in (m.linear_query.weight, m.linear_query.bias,
                                                               m.linear_key.weight, m.linear_relation.weight,
                                                               m.linear_relation.bias))
    Xd, dYd, QKd = X.to(dtype), dY.to(dtype), QK.to(dtype)
    G = dYd @ W_R
    S, dQ, dK = _edge_reference(src, dst, V, QKd[:, :H], QKd[:, H:], G, agg)
    return {"S": S, "dQ": dQ, "dK": dK, "Y": torch.addmm(b_R, S, W_R.t()), "dX": dQ @ W_Q + dK @ W_K,
            "dW_Q": dQ.t() @ Xd, "db_Q": dQ.sum(0), "dW_K": dK.t() @ Xd, "dW_R": dYd.t() @ S, "db_R": dYd.sum(0)}


def _per_tensor(got, r32, r64, what):
    e, e_ref = rel_err(got, r64), rel_err(r32, r64)
    assert e <= max(1e-5, 2 * e_ref), f"{what}: relL2 vs fp64 {e:.3e} > max(1e-5, 2 x ref32 {e_ref:.3e})"


@pytest.mark.timeout(400)
@pytest.mark.parametrize("agg", ["sum", "sym"])
def test_cfg4_S2_layer_deterministic_mask_equals_recompute_and_parity(s2, agg):
    g, X, dY = s2
    V = g.num_nodes()
    plan = get_plan(g, torch.device(DEV))
    assert plan.dst.n_splits > 0                                  # hub rows are split
    m, QK, a = _layer(g, X, dY, agg)
    _, QK2, b = _layer(g, X, dY, agg)
    assert torch.equal(QK, QK2)
    for k in a:
        assert torch.equal(a[k], b[k]), f"{agg} {k}: two runs differ"
    del b, QK2
    _, _, c = _layer(g, X, dY, agg, use_mask=False)                # recompute backward (no sign mask)
    for k in a:
        assert torch.equal(a[k], c[k]), f"{agg} {k}: sign-mask backward != recompute backward"
    del c
    # the QK GEMM against the fp64 projection
    W_cat = torch.cat([m.linear_query.weight, m.linear_key.weight], 0).detach().double()
    b_cat = torch.cat([m.linear_query.bias.detach(), torch.zeros(H, device=DEV)]).double()
    qk64 = torch.addmm(b_cat, X.double(), W_cat.t())
    qk32 = torch.addmm(b_cat.float(), X, W_cat.float().t())
    _per_tensor(QK, qk32, qk64, f"{agg} QK")
    del qk64, qk32, W_cat
    src, dst = g._src.to(DEV), g._dst.to(DEV)
    # the edge aggregation on the layer's own QK: S, dQ, dK (EdgeAggregate, the same kernels)
    x = QK.clone().requires_grad_(True)
    G = dY @ m.linear_relation.weight.detach()
    S = EdgeAggregate.apply(x, plan, H, agg, _native.ACT_LEAKY, 0.2)
    S.backward(G)
    torch.cuda.synchronize()
    r64 = _layer_reference(src, dst, V, X, QK, m, dY, agg, torch.float64)
    r32 = _layer_reference(src, dst, V, X, QK, m, dY, agg, torch.float32)
    for k, got in (("S", S.detach()), ("dQ", x.grad[:, :H]), ("dK", x.grad[:, H:])):
        _per_tensor(got, r32[k], r64[k], f"{agg} {k}")
    for k in a:
        _per_tensor(a[k], r32[k], r64[k], f"{agg} layer {k}")


@pytest.mark.timeout(600)
@pytest.mark.parametrize("agg", ["sum"])
def test_cfg4_S2_edge_cut_8_ranks_vs_single_gpu(s2, agg):
    """The edge-cut layer (sirgcn.dist, the scaling config: pipelined chunked exchanges, segmented
    forward) on the S2 graph over 8 ranks — one thread per rank on the one GPU (tests/thread_comm.py),
    every exchange on device tensors — run twice (bit-identical: fixed segment and peer orders), and
    Y, dX and the weight gradients (rank partials summed) per tensor against the fp64 reference on the
    single-GPU layer's projection values (the edge-cut's own QK equals it: the GEMMs are row-wise)."""
    from sirgcn.dist import DistGraph, DistSIRConvFunction, partition_rows
    from thread_comm import FakeCtx, ThreadComm, run_ranks
    g, X, dY = s2
    V = g.num_nodes()
    world = 8
    m, QK, one = _layer(g, X, dY, agg)
    w = [m.linear_query.weight.detach(), m.linear_query.bias.detach(), m.linear_key.weight.detach(),
         m.linear_relation.weight.detach(), m.linear_relation.bias.detach()]
    src, dst = g._src.to(DEV), g._dst.to(DEV)
    comms = ThreadComm.make(world)
    bounds = partition_rows(torch.bincount(dst, minlength=V), world)

    dgs = {}

    def fn(r):
        if r not in dgs:
            dgs[r] = DistGraph(src, dst, V, bounds, r, world, DEV, group=comms[r])
        dg = dgs[r]
        ctx = FakeCtx((True,) * 6 + (False,) * 7)
        sl = slice(dg.row_begin, dg.row_end)
        with torch.no_grad():
            Y = DistSIRConvFunction.forward(ctx, X[sl], *w, dg, agg, _native.ACT_LEAKY, 0.2, _native, True)
            grads = DistSIRConvFunction.backward(ctx, dY[sl])
        torch.cuda.synchronize()
        return dg.n_halo, Y, grads[:6]

    outs = run_ranks(world, fn)
    again = run_ranks(world, fn)
    for a, b in zip(outs, again):
        assert torch.equal(a[1], b[1]) and all(torch.equal(x, y) for x, y in zip(a[2], b[2]) if x is not None)
    del again
    assert all(o[0] > 0 for o in outs)
    got = {"Y": torch.cat([o[1] for o in outs]), "dX": torch.cat([o[2][0] for o in outs])}
    for i, k in enumerate(("dW_Q", "db_Q", "dW_K", "dW_R", "db_R"), start=1):
        got[k] = sum(o[2][i].double() for o in outs)
    del outs
    r64 = _layer_reference(src, dst, V, X, QK, m, dY, agg, torch.float64)
    r32 = _layer_reference(src, dst, V, X, QK, m, dY, agg, torch.float32)
    for k, v in got.items():
        _per_tensor(v, r32[k], r64[k], f"edge-cut x{world} {k}")

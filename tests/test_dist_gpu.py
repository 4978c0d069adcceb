"""Edge-cut layer (sirgcn.dist) on the GPU in one process, one thread per rank (tests/thread_comm.py):
the one-launch backward (``sir_edge_agg_bwd``: dQ and dK waves in one grid, then the reverse halo
exchange) and the autocast layer ``DistSIRConvFunction16`` (16-bit K_ext rows, edge passes and
both exchanges in the 16-bit storage type).

Tolerances: the one-launch backward is held BIT-EQUAL to the two-pass form (the same per-row
fp32 sums in the same order; MEAN divides G by the local in-degree first, as the single-GPU layer
does).  The 16-bit layer: relative L2 against the fp64 truth within 2e-2 (bf16) /
1e-2 (fp16), or no worse than 1.25x the reference's own AMP dataflow (``oracle.SIRConvRef`` under
the same autocast, single process) — the halo adds one 16-bit rounding per received dK row.
"""
import pytest
import torch
from torch import nn

import oracle
from conftest import rel_err

from sirgcn import _native
from sirgcn.conv import EdgeAggregate, SIRConv
from sirgcn.dist import (DistGraph, DistSIRConv, DistSIRConvFunction, DistSIRConvFunction16, _drop_at, _drops,
                         partition_rows)
from sirgcn.graph import Graph
from sirgcn.synth import powerlaw_edges
from thread_comm import FakeCtx, ThreadComm, run_ranks

pytestmark = pytest.mark.gpu
DEV = "cuda"
DT = {"bf16": torch.bfloat16, "f16": torch.float16}
TOL = {"bf16": 2e-2, "f16": 1e-2}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X box"
    _native.load()


def _problem(V, E, d, H, O, agg, seed=6):
    src, dst = powerlaw_edges(V, E, 0.8, seed=seed)
    X = torch.randn(V, d, generator=torch.Generator().manual_seed(1)).to(DEV)
    dY = torch.randn(V, O, generator=torch.Generator().manual_seed(2)).to(DEV)
    torch.manual_seed(3)
    conv = SIRConv(d, H, O, nn.LeakyReLU(0.2), 0, agg_type=agg).to(DEV)
    w = [conv.linear_query.weight.detach(), conv.linear_query.bias.detach(), conv.linear_key.weight.detach(),
         conv.linear_relation.weight.detach(), conv.linear_relation.bias.detach()]
    return src, dst, X, dY, conv, w


def _ranks(world, src, dst, V, fn):
    comms = ThreadComm.make(world)
    bounds = partition_rows(torch.bincount(dst, minlength=V), world)
    return run_ranks(world, lambda r: fn(r, DistGraph(src, dst, V, bounds, r, world, DEV, group=comms[r]),
                                         comms[r]))


@pytest.mark.parametrize("world,agg", [(2, "sum"), (3, "sym"), (2, "mean"), (4, "sum")])
def test_one_launch_backward_bit_equal_to_two_pass(world, agg, monkeypatch):
    V, E, H = 3000, 60000, 256   # sign-mask mode needs 128 < H (sir_mask_words)
    src, dst, X, dY, conv, w = _problem(V, E, H, H, H, agg)
    launches = []
    orig = _native.edge_agg_bwd

    def spy(*a, **k):
        launches.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(_native, "edge_agg_bwd", spy)

    def run(dual):
        monkeypatch.setattr(EdgeAggregate, "dual", dual)

        def fn(r, dg, comm):
            ctx = FakeCtx((True,) * 6 + (False,) * 7)
            sl = slice(dg.row_begin, dg.row_end)
            with torch.no_grad():
                Y = DistSIRConvFunction.forward(ctx, X[sl], *w, dg, agg, _native.ACT_LEAKY, 0.2, _native, True)
                g = DistSIRConvFunction.backward(ctx, dY[sl])
            torch.cuda.synchronize()
            return Y, g
        return _ranks(world, src, dst, V, fn)

    one = run(True)
    assert len(launches) == world                  # one sir_edge_agg_bwd per rank
    two = run(False)
    assert len(launches) == world
    for a, b in zip(one, two):
        assert torch.equal(a[0], b[0])
        for ga, gb in zip(a[1], b[1]):
            if ga is not None:
                assert torch.equal(ga, gb)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("world,agg", [(2, "sum"), (3, "sym"), (2, "mean")])
def test_autocast_edge_cut_16bit_wire(world, agg, dt):
    V, E, H = 3000, 60000, 256
    src, dst, X, dY, conv, w = _problem(V, E, H, H, H, agg, seed=8)
    wire = []

    def fn(r, dg, comm):
        orig = comm.all_to_all_rows

        def spy(out, inp, *a, **k):
            wire.append((out.dtype, inp.dtype))
            return orig(out, inp, *a, **k)
        comm.all_to_all_rows = spy
        ctx = FakeCtx((True,) * 6 + (False,) * 8)
        sl = slice(dg.row_begin, dg.row_end)
        with torch.no_grad():
            Y = DistSIRConvFunction16.forward(ctx, X[sl], *w, dg, agg, _native.ACT_LEAKY, 0.2, _native, True, True,
                                              DT[dt])
            g = DistSIRConvFunction16.backward(ctx, dY[sl])
        torch.cuda.synchronize()
        return dg.n_halo, Y, g

    outs = _ranks(world, src, dst, V, fn)
    assert all(o[0] > 0 for o in outs)
    rows = [(a, b) for a, b in wire if a.is_floating_point]      # (sym's plan-time out-degrees are int64)
    assert rows and all(a == DT[dt] and b == DT[dt] for a, b in rows)   # K rows out, dK rows back: 16-bit
    assert all(o[1].dtype == DT[dt] for o in outs)
    Y = torch.cat([o[1] for o in outs]).double().cpu()
    dX = torch.cat([o[2][0] for o in outs]).double().cpu()
    assert dX.dtype == torch.float64 and outs[0][2][0].dtype == torch.float32
    grads = [sum(o[2][i].double() for o in outs).cpu() for i in range(1, 6)]
    got = {"Y": Y, "dX": dX, **dict(zip(("dW_Q", "db_Q", "dW_K", "dW_R", "db_R"), grads))}
    _vs_amp_reference(got, conv, src, dst, V, X, dY, w, agg, DT[dt], TOL[dt])


def _vs_amp_reference(got, conv, src, dst, V, X, dY, w, agg, dt, tol):
    """relL2 vs fp64 within ``tol`` or 1.25x the reference's own AMP dataflow's error."""
    truth = oracle.layer_fwd_bwd(src, dst, V, X.cpu().double(), *[t.cpu().double() for t in w],
                                 dY.cpu().double(), agg, "leaky", 0.2)
    H = w[0].shape[0]
    ref = oracle.SIRConvRef(X.shape[1], H, w[3].shape[0], nn.LeakyReLU(0.2), 0, agg_type=agg).to(DEV)
    ref.load_state_dict(conv.state_dict())
    xr = X.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=dt):
        Yr = ref(Graph(src, dst, V), xr)
    Yr.backward(dY.to(Yr.dtype))
    amp = {"Y": Yr, "dX": xr.grad, "dW_Q": ref.linear_query.weight.grad, "db_Q": ref.linear_query.bias.grad,
           "dW_K": ref.linear_key.weight.grad, "dW_R": ref.linear_relation.weight.grad,
           "db_R": ref.linear_relation.bias.grad}
    for k, v in got.items():
        e, e_amp = rel_err(v.double().cpu(), truth[k]), rel_err(amp[k].double().cpu(), truth[k])
        assert e <= max(tol, 1.25 * e_amp), (k, e, e_amp)


def test_dist_layer_routes_autocast_to_the_16bit_function(monkeypatch):
    """DistSIRConv.forward under autocast takes DistSIRConvFunction16 (world 1: no exchange) and
    its gradients flow through Tensor.backward."""
    V, E, H = 2000, 30000, 128
    src, dst, X, dY, conv, w = _problem(V, E, H, H, H, "sym")
    calls = []
    orig = DistSIRConvFunction16.apply
    monkeypatch.setattr(DistSIRConvFunction16, "apply", staticmethod(lambda *a: calls.append(1) or orig(*a)))
    dg = DistGraph.from_global(src, dst, V, 0, 1, DEV)
    layer = DistSIRConv(conv)
    xr = X.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        Y = layer(dg, xr)
    Y.backward(dY.to(Y.dtype))
    assert calls == [1] and Y.dtype == torch.bfloat16 and xr.grad.dtype == torch.float32
    got = {"Y": Y.detach(), "dX": xr.grad, "dW_Q": conv.linear_query.weight.grad,
           "db_Q": conv.linear_query.bias.grad, "dW_K": conv.linear_key.weight.grad,
           "dW_R": conv.linear_relation.weight.grad, "db_R": conv.linear_relation.bias.grad}
    _vs_amp_reference({k: v.clone() for k, v in got.items()}, conv, src, dst, V, X, dY, w, "sym",
                      torch.bfloat16, 2e-2)


@pytest.mark.parametrize("world,agg", [(3, "sum"), (2, "sym")])
def test_edge_cut_training_dropout_vs_explicit_mask(world, agg):
    """Training-mode feature dropout in the fused edge-cut function (conv.py:35,60-61; the reference
    trains with p = 0.2, ogbn-arxiv/train.py:303): Q and K masks from two device seeds per rank in
    the GEMM epilogues, the owners' masks applied to dQ / dK after the exchange — against the
    reference dataflow with the same masks applied explicitly (fp32 reference and fp64 truth)."""
    from conftest import assert_parity
    V, E, H = 2500, 50000, 256
    p = 0.2
    src, dst, X, dY, conv, w = _problem(V, E, 64, H, 32, agg, seed=11)
    comms = ThreadComm.make(world)
    bounds = partition_rows(torch.bincount(dst, minlength=V), world)
    seeds = [torch.tensor([1000 + 2 * r, 1001 + 2 * r], device=DEV) for r in range(world)]

    def fn(r):
        dg = DistGraph(src, dst, V, bounds, r, world, DEV, group=comms[r])
        ctx = FakeCtx((True,) * 6 + (False,) * 8)
        sl = slice(dg.row_begin, dg.row_end)
        with torch.no_grad():
            Y = DistSIRConvFunction.forward(ctx, X[sl], *w, dg, agg, _native.ACT_LEAKY, 0.2, _native, True, True,
                                            (seeds[r], p))
            g = DistSIRConvFunction.backward(ctx, dY[sl])
        torch.cuda.synchronize()
        n = dg.n_rows
        # the masks the layer drew: seeds offset by the rank's first row (Q, K) and, for K (projected part
        # by part), by the part's first row
        dq, dk = _drops((seeds[r], p), dg.row_begin)
        mq = _native.dropout_apply(torch.ones(n, H, device=DEV), dq)
        mk = torch.ones(n, H, device=DEV)
        for c in range(dg.chunks):
            a, b = dg.own_range(c)
            if b > a:
                _native.dropout_apply(mk[a:b], _drop_at(dk, a))
        return Y, g, mq, mk

    outs = run_ranks(world, fn)
    Mk = torch.cat([torch.cat([o[2], o[3]], 1) for o in outs]).cpu()
    assert 0.15 < float((Mk == 0).float().mean()) < 0.25
    # equal local rows of two ranks draw different bits
    assert not torch.equal(outs[0][2][:64].cpu(), outs[1][2][:64].cpu())
    got = {"Y": torch.cat([o[0] for o in outs]).cpu(), "dX": torch.cat([o[1][0] for o in outs]).cpu()}
    for i, k in enumerate(("dW_Q", "db_Q", "dW_K", "dW_R", "db_R"), start=1):
        got[k] = sum(o[1][i].double() for o in outs).cpu()

    def ref(dtype):
        t = lambda x: x.detach().cpu().to(dtype).requires_grad_(True)
        X64, WQ, bQ, WK, WR, bR = (t(x) for x in (X, *w))
        M = Mk.to(dtype)
        Q = (X64 @ WQ.t() + bQ) * M[:, :H]
        K = (X64 @ WK.t()) * M[:, H:]
        S = oracle.edge_agg_fwd(src, dst, V, Q, K, agg, "leaky", 0.2)
        Y = S @ WR.t() + bR
        Y.backward(dY.cpu().to(dtype))
        return {"Y": Y.detach(), "dX": X64.grad, "dW_Q": WQ.grad, "db_Q": bQ.grad, "dW_K": WK.grad,
                "dW_R": WR.grad, "db_R": bR.grad}
    r32, r64 = ref(torch.float32), ref(torch.float64)
    for k, v in got.items():
        assert_parity(v, r32[k], r64[k], 1e-5, f"edge-cut dropout x{world} {agg} {k}", strict=(k == "Y"))


@pytest.mark.parametrize("world", [2, 3])
def test_edge_cut_max_vs_single_gpu(world):
    """agg_type='max' on the edge-cut (conv.py:46-47 + fn.max): own-row Q, K_ext = [own | halo] K rows
    gathered by the chunked alltoallv (HaloGather), the fused per-edge W_R with the running max on them
    (EdgeMaxLinearQK), the halo rows' dK sent back to their owners — against the single-GPU layer with
    the same weights.  The GEMMs are row-wise, so every Q / K row is the single-GPU value: Y is held to
    1e-6.  The ranks are threads on the one GPU; their backward runs through the Functions' own
    backward (the autograd engine has one worker per device: concurrent Tensor.backward calls of
    threads that exchange rows would deadlock on it)."""
    from sirgcn.dist import HaloGather
    from sirgcn.edgemlp import EdgeMaxLinearQK
    V, E, H, O = 3000, 60000, 128, 64
    src, dst = powerlaw_edges(V, E, 0.8, seed=21)
    X = torch.randn(V, 48, generator=torch.Generator().manual_seed(1)).to(DEV)
    dY = torch.randn(V, O, generator=torch.Generator().manual_seed(2)).to(DEV)
    torch.manual_seed(4)
    conv = SIRConv(48, H, O, nn.LeakyReLU(0.2), 0, agg_type="max").to(DEV)
    xs = X.clone().requires_grad_(True)
    Ys = conv(Graph(src, dst, V), xs)
    Ys.backward(dY)
    ref = {"Y": Ys.detach(), "dX": xs.grad, "dW_Q": conv.linear_query.weight.grad, "db_Q": conv.linear_query.bias.grad,
           "dW_K": conv.linear_key.weight.grad, "dW_R": conv.linear_relation.weight.grad,
           "db_R": conv.linear_relation.bias.grad}
    WQ, bQ, WK = conv.linear_query.weight.detach(), conv.linear_query.bias.detach(), conv.linear_key.weight.detach()
    WR, bR = conv.linear_relation.weight.detach(), conv.linear_relation.bias.detach()
    comms = ThreadComm.make(world)
    bounds = partition_rows(torch.bincount(dst.to(DEV), minlength=V), world)

    def fn(r):
        dg = DistGraph(src, dst, V, bounds, r, world, DEV, group=comms[r])
        sl = slice(dg.row_begin, dg.row_end)
        x = X[sl]
        with torch.no_grad():
            Q = x @ WQ.t() + bQ
            K = x @ WK.t()
            c1, c2 = FakeCtx((True, False)), FakeCtx((True, True, True, True, False, False, False))
            K_ext = HaloGather.forward(c1, K, dg)
            Y = EdgeMaxLinearQK.forward(c2, Q, K_ext, WR, bR, dg, _native.ACT_LEAKY, 0.2)
            dQ, dK_ext, dWR, dbR = EdgeMaxLinearQK.backward(c2, dY[sl])[:4]
            dK = HaloGather.backward(c1, dK_ext)[0]
        torch.cuda.synchronize()
        return {"Y": Y, "dX": dQ @ WQ + dK @ WK, "dW_Q": dQ.t() @ x, "db_Q": dQ.sum(0), "dW_K": dK.t() @ x,
                "dW_R": dWR, "db_R": dbR}

    outs = run_ranks(world, fn)
    got = {k: torch.cat([o[k] for o in outs]) for k in ("Y", "dX")}
    for k in ("dW_Q", "db_Q", "dW_K", "dW_R", "db_R"):
        got[k] = sum(o[k].double() for o in outs).float()
    for k, v in got.items():
        e = float((v.double() - ref[k].double()).norm() / ref[k].double().norm().clamp_min(1e-30))
        assert e < (1e-6 if k == "Y" else 1e-5), (k, e)


def test_edge_cut_max_training_dropout_hashed_per_rank():
    """agg_type='max' on the edge-cut in training mode: Q / K dropout is the hashed mask of the
    layer's two device seeds mixed with the rank's first global row (advisor r05: the module's
    nn.Dropout gave ranks seeded alike identical masks for their local rows).  World 1: the layer
    equals the explicit chain with those masks, forward and every gradient, bit for bit; a rank
    starting at another row draws different bits."""
    from sirgcn.dist import HaloGather, HashedDropout
    from sirgcn.edgemlp import EdgeMaxLinearQK
    V, E, H, O, p = 2000, 30000, 128, 64, 0.2
    src, dst = powerlaw_edges(V, E, 0.8, seed=23)
    X = torch.randn(V, 48, generator=torch.Generator().manual_seed(1)).to(DEV)
    dY = torch.randn(V, O, generator=torch.Generator().manual_seed(2)).to(DEV)
    torch.manual_seed(4)
    conv = SIRConv(48, H, O, nn.LeakyReLU(0.2), p, agg_type="max").to(DEV).train()
    dg = DistGraph.from_global(src, dst, V, 0, 1, DEV)
    layer = DistSIRConv(conv)
    xr = X.clone().requires_grad_(True)
    torch.cuda.manual_seed(77)
    Y = layer(dg, xr)
    Y.backward(dY)
    got = [Y.detach(), xr.grad] + [q.grad.clone() for q in conv.parameters()]
    torch.cuda.manual_seed(77)
    seeds = torch.randint(0, 2 ** 62, (2,), device=DEV, dtype=torch.int64)
    dq, dk = _drops((seeds, p), dg.row_begin)
    mq = _native.dropout_apply(torch.ones(V, H, device=DEV), dq)
    assert 0.15 < float((mq == 0).float().mean()) < 0.25
    other = _native.dropout_apply(torch.ones(V, H, device=DEV), _drops((seeds, p), 1000)[0])
    assert not torch.equal(mq, other)
    for q in conv.parameters():
        q.grad = None
    xe = X.clone().requires_grad_(True)
    Q = HashedDropout.apply(conv._linear(xe, conv.linear_query.weight, conv.linear_query.bias), dq)
    K = HashedDropout.apply(conv._linear(xe, conv.linear_key.weight, None), dk)
    assert torch.equal(Q.detach() == 0, (mq == 0) | (Q.detach() == 0))
    Ye = EdgeMaxLinearQK.apply(Q, HaloGather.apply(K, dg), conv.linear_relation.weight, conv.linear_relation.bias,
                               dg, _native.ACT_LEAKY, 0.2)
    Ye.backward(dY)
    want = [Ye.detach(), xe.grad] + [q.grad for q in conv.parameters()]
    for a, b in zip(got, want):
        assert torch.equal(a, b)

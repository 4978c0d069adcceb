"""Multi-rank edge-cut (sirgcn.dist) on CPU with gloo, world sizes 2-4: partition invariants,
the sparse halo all-to-all (forward K rows) and its transpose (backward dK rows), the weight-gradient
all-reduce, and the assembled layer
output + gradients against the single-process CPU oracle.  The per-rank edge math uses the
test-only CPU backend (tests/cpu_edge_backend.py); the GPU path is covered by -m gpu tests."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT, assert_close


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, agg, outdir, fused=True, chunks=None, reduce=False):
    for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from torch import nn
    import cpu_edge_backend
    from sirgcn import SIRConv
    from sirgcn.dist import DistGraph, DistSIRConv
    from sirgcn.synth import powerlaw_edges
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    V, E, d, H, O = 500, 6000, 16, 40, 12
    src, dst = powerlaw_edges(V, E, 0.8, seed=7)
    X = torch.randn(V, d, generator=torch.Generator().manual_seed(1))
    dY = torch.randn(V, O, generator=torch.Generator().manual_seed(2))
    torch.manual_seed(3)
    conv = SIRConv(d, H, O, nn.LeakyReLU(0.2), 0, agg_type=agg)
    dg = DistGraph.from_global(src, dst, V, rank, world, "cpu", chunk=64, chunks=chunks)
    dconv = DistSIRConv(conv, backend=cpu_edge_backend, reduce_in_backward=reduce)
    dconv.use_fused = fused
    r0, r1 = dg.row_begin, dg.row_end
    Xl = X[r0:r1].clone().requires_grad_(True)
    Y = dconv(dg, Xl)
    Y.backward(dY[r0:r1])
    dconv.allreduce_grads()
    torch.save({"r0": r0, "r1": r1, "Y": Y.detach(), "dX": Xl.grad, "E_local": dg.num_local_edges,
                "bounds": dg.bounds, "grads": {n: p.grad for n, p in conv.named_parameters()},
                "halo": dg.halo_ids, "recv_splits": dg.recv_splits, "send_splits": dg.send_splits,
                "send_idx": dg.send_idx, "halo_off": dg.halo_off, "out_deg": dg.out_deg()},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,agg,fused,chunks,reduce", [(2, "sum", True, None, False), (2, "sym", True, 1, False),
                                                           (3, "mean", True, 3, False), (4, "sym", True, None, False),
                                                           (3, "sum", False, 2, False), (2, "mean", False, 7, False),
                                                           (3, "sum", True, 4, True), (2, "sym", True, 2, True)])
def test_edge_cut_matches_single_process_oracle(tmp_path, world, agg, fused, chunks, reduce):
    """``reduce``: the weight gradients are all-reduced inside the fused backward (dW_R / dW_Q under the
    reverse exchange, dW_K last); allreduce_grads() must then leave them alone."""
    import oracle
    from sirgcn.synth import powerlaw_edges
    from torch import nn
    from sirgcn import SIRConv
    mp.spawn(_worker, args=(world, _free_port(), agg, str(tmp_path), fused, chunks, reduce), nprocs=world, join=True)
    parts = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    V, E, d, H, O = 500, 6000, 16, 40, 12
    src, dst = powerlaw_edges(V, E, 0.8, seed=7)
    X = torch.randn(V, d, generator=torch.Generator().manual_seed(1))
    dY = torch.randn(V, O, generator=torch.Generator().manual_seed(2))
    torch.manual_seed(3)
    conv = SIRConv(d, H, O, nn.LeakyReLU(0.2), 0, agg_type=agg)
    w = [conv.linear_query.weight, conv.linear_query.bias, conv.linear_key.weight,
         conv.linear_relation.weight, conv.linear_relation.bias]
    ref = oracle.reference_cpu_step(src, dst, V, X, *[t.detach() for t in w], dY, agg, "leaky", 0.2)
    # partition covers all rows / edges exactly once, contiguous, edge-balanced
    assert parts[0]["r0"] == 0 and parts[-1]["r1"] == V
    assert all(parts[i]["r1"] == parts[i + 1]["r0"] for i in range(world - 1))
    assert sum(p["E_local"] for p in parts) == E
    assert max(p["E_local"] for p in parts) <= E / world + int(torch.bincount(dst, minlength=V).max())
    # halo exchange plan: every rank's halo = its distinct remote sources, stored chunk-major (each
    # chunk: a part of every owner's block, owners in order); what owner q sends to rank p in chunk c
    # is exactly p's chunk-c slice owned by q, in the same order
    C = len(parts[0]["recv_splits"])
    assert C == (chunks if chunks is not None else 4)
    for p, part in enumerate(parts):
        r0, r1 = part["r0"], part["r1"]
        sel = (dst >= r0) & (dst < r1)
        s_ = src[sel]
        want = torch.unique(s_[(s_ < r0) | (s_ >= r1)])
        assert torch.equal(torch.sort(part["halo"]).values, want)
        for c in range(C):
            off = part["halo_off"][c]
            for q in range(world):
                n = part["recv_splits"][c][q]
                mine = part["halo"][off:off + n]
                off += n
                if n:
                    assert int(mine.min()) >= parts[q]["r0"] and int(mine.max()) < parts[q]["r1"]
                    assert torch.all(mine[1:] > mine[:-1])
                so = sum(parts[q]["send_splits"][c][:p])
                sent = parts[q]["send_idx"][c][so:so + parts[q]["send_splits"][c][p]] + parts[q]["r0"]
                assert torch.equal(sent, mine)
            assert off == part["halo_off"][c + 1]
        # global out-degree of own + halo rows
        gdeg = torch.bincount(src, minlength=V)
        ext = torch.cat([torch.arange(r0, r1), part["halo"]])
        assert torch.equal(part["out_deg"], gdeg[ext])
    Y = torch.cat([p["Y"] for p in parts])
    dX = torch.cat([p["dX"] for p in parts])
    assert_close(Y, ref["Y"], 1e-5, "Y")
    assert_close(dX, ref["dX"], 1e-5, "dX")
    names = {"linear_query.weight": "dW_Q", "linear_query.bias": "db_Q", "linear_key.weight": "dW_K",
             "linear_relation.weight": "dW_R", "linear_relation.bias": "db_R"}
    for p in parts:   # every rank holds the same all-reduced weight gradients
        for n, k in names.items():
            assert_close(p["grads"][n], ref[k], 1e-5, f"{n}")


@pytest.mark.parametrize("row_weight", [0, 12])
def test_partition_rows_balances_cost(row_weight):
    """Contiguous row ranges with equal cost = in-edges + row_weight per row, to within one row."""
    from sirgcn.dist import partition_rows
    from sirgcn.synth import powerlaw_edges
    V, E = 10_000, 200_000
    _, dst = powerlaw_edges(V, E, 0.8, seed=1)
    deg = torch.bincount(dst, minlength=V)
    cost = deg + row_weight
    total = int(cost.sum())
    for world in (1, 2, 4, 8):
        b = partition_rows(deg, world, row_weight=row_weight)
        assert b[0] == 0 and b[-1] == V and all(b[i] <= b[i + 1] for i in range(world))
        loads = [int(cost[b[i]:b[i + 1]].sum()) for i in range(world)]
        assert sum(loads) == total
        assert max(loads) <= total / world + int(cost.max())


@pytest.mark.parametrize("world,agg", [(2, "sum"), (3, "sym"), (4, "mean")])
def test_edge_cut_fused_function_threads(world, agg):
    """DistSIRConvFunction driven by hand on one thread per rank (tests/thread_comm.py), the
    same harness the -m gpu test uses on device tensors, here with the CPU edge backend."""
    import cpu_edge_backend
    import oracle
    from torch import nn
    from conftest import assert_parity
    from sirgcn import SIRConv, _native
    from sirgcn.dist import DistGraph, DistSIRConvFunction, partition_rows
    from sirgcn.synth import powerlaw_edges
    from thread_comm import FakeCtx, ThreadComm, run_ranks
    V, E, H = 600, 9000, 24
    src, dst = powerlaw_edges(V, E, 0.8, seed=6)
    X = torch.randn(V, 16, generator=torch.Generator().manual_seed(1))
    dY = torch.randn(V, 8, generator=torch.Generator().manual_seed(2))
    torch.manual_seed(3)
    conv = SIRConv(16, H, 8, nn.LeakyReLU(0.2), 0, agg_type=agg)
    w = [p.detach() for p in (conv.linear_query.weight, conv.linear_query.bias, conv.linear_key.weight,
                              conv.linear_relation.weight, conv.linear_relation.bias)]
    comms = ThreadComm.make(world)
    bounds = partition_rows(torch.bincount(dst, minlength=V), world)

    def fn(r):
        dg = DistGraph(src, dst, V, bounds, r, world, "cpu", chunk=64, group=comms[r])
        ctx = FakeCtx((True,) * 6 + (False,) * 7)
        Y = DistSIRConvFunction.forward(ctx, X[dg.row_begin:dg.row_end], *w, dg, agg, _native.ACT_LEAKY, 0.2,
                                        cpu_edge_backend, True)
        return dg.n_halo, Y, DistSIRConvFunction.backward(ctx, dY[dg.row_begin:dg.row_end])

    outs = run_ranks(world, fn)
    assert all(o[0] > 0 for o in outs)
    Y = torch.cat([o[1] for o in outs])
    dX = torch.cat([o[2][0] for o in outs])
    t = oracle.layer_fwd_bwd(src, dst, V, X.double(), *[x.double() for x in w], dY.double(), agg, "leaky", 0.2)
    r = oracle.reference_cpu_step(src, dst, V, X, *w, dY, agg, "leaky", 0.2)
    assert_parity(Y, r["Y"], t["Y"], 1e-5, "Y")
    assert_parity(dX, r["dX"], t["dX"], 1e-5, "dX")
    for i, k in enumerate(("dW_Q", "db_Q", "dW_K", "dW_R", "db_R")):
        assert_parity(sum(o[2][i + 1] for o in outs), r[k], t[k], 1e-5, k)


@pytest.mark.parametrize("agg", ["sum", "mean"])
def test_edge_cut_async_exchange_waits_before_use(agg):
    """The async all-to-all path of DistSIRConvFunction (async_op=True, work.wait()) with a group
    whose rows arrive only at wait() (NaN before): the assembled result must still match the oracle."""
    import cpu_edge_backend
    import oracle
    from torch import nn
    from conftest import assert_parity
    from sirgcn import SIRConv, _native
    from sirgcn.dist import DistGraph, DistSIRConvFunction, partition_rows
    from sirgcn.synth import powerlaw_edges
    from thread_comm import DeferredComm, FakeCtx, run_ranks
    world, V, E, H = 3, 500, 7000, 16
    src, dst = powerlaw_edges(V, E, 0.8, seed=9)
    X = torch.randn(V, 12, generator=torch.Generator().manual_seed(1))
    dY = torch.randn(V, 8, generator=torch.Generator().manual_seed(2))
    torch.manual_seed(3)
    conv = SIRConv(12, H, 8, nn.LeakyReLU(0.2), 0, agg_type=agg)
    w = [p.detach() for p in (conv.linear_query.weight, conv.linear_query.bias, conv.linear_key.weight,
                              conv.linear_relation.weight, conv.linear_relation.bias)]
    comms = DeferredComm.make(world)
    bounds = partition_rows(torch.bincount(dst, minlength=V), world)

    def fn(r):
        dg = DistGraph(src, dst, V, bounds, r, world, "cpu", chunk=64, group=comms[r])
        ctx = FakeCtx((True,) * 6 + (False,) * 7)
        Y = DistSIRConvFunction.forward(ctx, X[dg.row_begin:dg.row_end], *w, dg, agg, _native.ACT_LEAKY, 0.2,
                                        cpu_edge_backend, True)
        return Y, DistSIRConvFunction.backward(ctx, dY[dg.row_begin:dg.row_end]), comms[r].works

    outs = run_ranks(world, fn)
    assert all(o[2] == 8 for o in outs)          # four async chunk exchanges forward, four backward, per rank
    Y = torch.cat([o[0] for o in outs])
    dX = torch.cat([o[1][0] for o in outs])
    assert torch.isfinite(Y).all() and torch.isfinite(dX).all()
    t = oracle.layer_fwd_bwd(src, dst, V, X.double(), *[x.double() for x in w], dY.double(), agg, "leaky", 0.2)
    r = oracle.reference_cpu_step(src, dst, V, X, *w, dY, agg, "leaky", 0.2)
    assert_parity(Y, r["Y"], t["Y"], 1e-5, "Y")
    assert_parity(dX, r["dX"], t["dX"], 1e-5, "dX")


def _dropout_worker(rank, world, port, outdir):
    for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from torch import nn
    import cpu_edge_backend
    from sirgcn import SIRConv
    from sirgcn.dist import DistGraph, DistSIRConv
    from sirgcn.synth import powerlaw_edges
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    V, E, d, H, O = 300, 3000, 8, 16, 8
    src, dst = powerlaw_edges(V, E, 0.8, seed=5)
    X = torch.randn(V, d, generator=torch.Generator().manual_seed(1))
    torch.manual_seed(3)
    conv = SIRConv(d, H, O, nn.ReLU(), 0.5, agg_type="sum")
    conv.train()
    dg = DistGraph.from_global(src, dst, V, rank, world, "cpu", chunk=64)
    dconv = DistSIRConv(conv, backend=cpu_edge_backend)       # use_fused stays True: CPU + p > 0 must not enter it
    r0, r1 = dg.row_begin, dg.row_end
    Xl = X[r0:r1].clone().requires_grad_(True)
    Y = dconv(dg, Xl)
    Y.sum().backward()
    dconv.allreduce_grads()
    torch.save({"Y": Y.detach(), "dX": Xl.grad, "gq": conv.linear_query.weight.grad}, os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_edge_cut_training_dropout_on_cpu_takes_the_modular_path(tmp_path):
    """CPU rehearsals with dropout > 0 in train mode must not reach the native dropout
    kernels (host pointers); they run nn.Dropout on the modular path."""
    mp.spawn(_dropout_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        part = torch.load(tmp_path / f"rank{r}.pt", weights_only=True)
        assert torch.isfinite(part["Y"]).all() and torch.isfinite(part["dX"]).all()
        assert part["gq"] is not None and torch.isfinite(part["gq"]).all()


def test_dropout_seeds_differ_across_ranks():
    """the kernels hash the LOCAL row index, so each rank's seeds are offset by its first
    global row; rank 0 (row_begin 0) keeps the drawn seeds."""
    sys.path.insert(0, PKG)
    from sirgcn.dist import _drops
    seeds = torch.tensor([123456789, 987654321], dtype=torch.int64)
    q0, k0 = _drops((seeds, 0.2), 0)
    q1, k1 = _drops((seeds, 0.2), 1000)
    assert int(q0[0]) == 123456789 and int(k0[0]) == 987654321
    assert int(q1[0]) != int(q0[0]) and int(k1[0]) != int(k0[0])
    a, b = _drops((42, 0.2), 0), _drops((42, 0.2), 77)
    assert a[0][0] == 42 and a[0][0] != b[0][0] and a[1][0] != b[1][0]


@pytest.mark.parametrize("agg", ["sum", "sym"])
def test_single_process_reduce_in_backward_without_process_group(agg):
    """``DistSIRConv(reduce_in_backward=True)`` on one process with no process group (world 1, no halo
    chunks): the in-backward reducer has nothing to reduce, as ``allreduce_grads`` (advisor r05 finding);
    layer output and every gradient match the CPU oracle."""
    import torch.distributed as dist
    import oracle
    from torch import nn
    import cpu_edge_backend
    from sirgcn import SIRConv
    from sirgcn.dist import DistGraph, DistSIRConv
    from sirgcn.synth import powerlaw_edges
    assert not dist.is_initialized()
    V, E, d, H, O = 300, 3000, 16, 40, 12
    src, dst = powerlaw_edges(V, E, 0.8, seed=7)
    X = torch.randn(V, d, generator=torch.Generator().manual_seed(1))
    dY = torch.randn(V, O, generator=torch.Generator().manual_seed(2))
    torch.manual_seed(3)
    conv = SIRConv(d, H, O, nn.LeakyReLU(0.2), 0, agg_type=agg)
    dg = DistGraph.from_global(src, dst, V, 0, 1, "cpu", chunk=64)
    dconv = DistSIRConv(conv, backend=cpu_edge_backend, reduce_in_backward=True)
    Xl = X.clone().requires_grad_(True)
    Y = dconv(dg, Xl)
    Y.backward(dY)
    dconv.allreduce_grads()
    w = [conv.linear_query.weight, conv.linear_query.bias, conv.linear_key.weight,
         conv.linear_relation.weight, conv.linear_relation.bias]
    ref = oracle.reference_cpu_step(src, dst, V, X, *[t.detach() for t in w], dY, agg, "leaky", 0.2)
    assert_close(Y.detach(), ref["Y"], 1e-5, "Y")
    assert_close(Xl.grad, ref["dX"], 1e-5, "dX")
    for p, k in zip(w, ("dW_Q", "db_Q", "dW_K", "dW_R", "db_R")):
        assert_close(p.grad, ref[k], 1e-5, k)

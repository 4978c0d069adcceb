"""cfg5's data-parallel step (``bench.py --gpus N --workload cfg5``: ``workloads.dp_replica`` +
DDP) rehearsed on CPU with gloo, world sizes 2 and 3: each rank holds its own batch of molecules
and the replicated 5-layer SIRConv/GraphNorm stack; after one backward every rank must hold the
AVERAGE of the per-batch gradients (DDP's all-reduce / world) and identical weights.  The stack is
built on the oracle's restated modules (the same classes the -m gpu stack tests compare against),
since the product layer has no CPU path; the DP plumbing under test is the product's.

Tolerance: 1e-5 relative (fp32 all-reduce of world terms vs a float64 average of the same fp32
per-batch gradients); the analytically-zero db_R behind GraphNorm: 64 * 2^-24 * sum_v |dL/dY_conv[v]|."""
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


def _worker(rank, world, port, outdir):
    for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    import oracle
    from sirgcn.workloads import dp_replica
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    model, stack, g, X, dY = dp_replica("cfg5", rank, world, torch.device("cpu"), oracle.SIRConvRef,
                                        oracle.GraphNormRef, small=True)
    assert isinstance(model, torch.nn.parallel.DistributedDataParallel)
    Y = model(g, X)
    Y.backward(dY)
    torch.save({"grads": {n: p.grad for n, p in stack.named_parameters() if p.grad is not None},
                "E": g.num_edges(), "V": g.num_nodes()}, os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_cfg5_data_parallel_gradients_are_the_batch_average(tmp_path, world):
    import oracle
    from sirgcn.workloads import dp_replica
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    parts = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    assert len({p["E"] for p in parts}) > 1 or len({p["V"] for p in parts}) > 1   # a different batch per rank
    local = []
    for r in range(world):      # each rank's batch alone, single process (world 1: no DDP)
        model, stack, g, X, dY = dp_replica("cfg5", r, 1, torch.device("cpu"), oracle.SIRConvRef,
                                            oracle.GraphNormRef, small=True)
        assert model is stack
        gsum = {}
        for i, conv in enumerate(stack.convs):   # sum_v |dL/dY_conv[v]|: the terms db_R sums
            conv.linear_relation.register_full_backward_hook(
                lambda mod, gin, gout, i=i: gsum.__setitem__(f"convs.{i}.linear_relation.bias",
                                                             gout[0].detach().abs().sum(0).double()))
        model(g, X).backward(dY)
        local.append(({n: p.grad.double() for n, p in stack.named_parameters() if p.grad is not None}, gsum))
    for n in local[0][0]:
        avg = sum(l[0][n] for l in local) / world
        if n in local[0][1]:
            scale = sum(l[1][n] for l in local) / world
            if avg.norm() <= 1e-5 * scale.norm():
                # linear_relation.bias behind GraphNorm: analytically 0 (the norm removes any
                # per-feature constant), each batch's value is rounding noise of a sum of V terms
                # (its order differs with the thread count): absolute bound 64 u sum|terms|
                for p in parts:
                    assert torch.all((p["grads"][n].double() - avg).abs() <= 64 * 2.0 ** -24 * scale), n
                continue
        for p in parts:
            assert_close(p["grads"][n].double(), avg, 1e-5, n)

"""The edge-cut layer over real RCCL (``torch.distributed`` backend "nccl" = RCCL on ROCm), one
process per GPU — the launch ``bench.py --gpus N`` uses.  Skipped on boxes with fewer than two
GPUs (the per-round GPU box has one; the driver's 8-GPU node runs the bench).  The same layer is
covered on one GPU by the threaded tests (test_dist_gpu.py, test_gpu_parity.py) and on CPU with
gloo (test_dist_gloo.py).

Tolerances as there: fp32 through ``assert_parity`` (1e-5 relative, or no worse than twice the
fp32 reference's error against fp64); bf16 autocast relative L2 within 2e-2 of the fp64 truth."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT, assert_parity, rel_err

pytestmark = pytest.mark.gpu
NGPU = torch.cuda.device_count()
V, E, H = 4000, 80000, 256      # > 128: the sign-mask (one-launch backward) mode


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, agg, autocast, outdir):
    for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from torch import nn
    from sirgcn import SIRConv, _native
    from sirgcn.dist import DistGraph, DistSIRConv
    from sirgcn.synth import powerlaw_edges
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    _native.load()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            device_id=dev)
    src, dst = powerlaw_edges(V, E, 0.8, seed=6)
    X = torch.randn(V, H, generator=torch.Generator().manual_seed(1))
    dY = torch.randn(V, H, generator=torch.Generator().manual_seed(2))
    torch.manual_seed(3)
    conv = SIRConv(H, H, H, nn.LeakyReLU(0.2), 0, agg_type=agg).to(dev)
    dg = DistGraph.from_global(src, dst, V, rank, world, dev)
    layer = DistSIRConv(conv)
    r0, r1 = dg.row_begin, dg.row_end
    x = X[r0:r1].to(dev).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        Y = layer(dg, x)
    Y.backward(dY[r0:r1].to(dev, Y.dtype))
    layer.allreduce_grads()
    torch.cuda.synchronize()
    torch.save({"Y": Y.detach().float().cpu(), "dX": x.grad.cpu(), "halo": dg.n_halo,
                "grads": {n: p.grad.cpu() for n, p in conv.named_parameters()}},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.skipif(NGPU < 2, reason="needs >= 2 GPUs (RCCL over xGMI)")
@pytest.mark.parametrize("agg,autocast", [("sum", False), ("sym", False), ("mean", False), ("sym", True)])
def test_edge_cut_over_rccl(tmp_path, agg, autocast):
    import oracle
    from torch import nn
    from sirgcn import SIRConv
    from sirgcn.synth import powerlaw_edges
    world = min(NGPU, 8)
    mp.spawn(_worker, args=(world, _free_port(), agg, autocast, str(tmp_path)), nprocs=world, join=True)
    parts = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    assert sum(p["halo"] for p in parts) > 0
    src, dst = powerlaw_edges(V, E, 0.8, seed=6)
    X = torch.randn(V, H, generator=torch.Generator().manual_seed(1))
    dY = torch.randn(V, H, generator=torch.Generator().manual_seed(2))
    torch.manual_seed(3)
    conv = SIRConv(H, H, H, nn.LeakyReLU(0.2), 0, agg_type=agg)
    w = [p.detach() for p in (conv.linear_query.weight, conv.linear_query.bias, conv.linear_key.weight,
                              conv.linear_relation.weight, conv.linear_relation.bias)]
    t = oracle.layer_fwd_bwd(src, dst, V, X.double(), *[x.double() for x in w], dY.double(), agg, "leaky", 0.2)
    Y = torch.cat([p["Y"] for p in parts])
    dX = torch.cat([p["dX"] for p in parts])
    names = {"linear_query.weight": "dW_Q", "linear_query.bias": "db_Q", "linear_key.weight": "dW_K",
             "linear_relation.weight": "dW_R", "linear_relation.bias": "db_R"}
    if autocast:
        assert rel_err(Y.double(), t["Y"]) <= 2e-2 and rel_err(dX.double(), t["dX"]) <= 2e-2
        for p in parts:
            for n, k in names.items():
                assert rel_err(p["grads"][n].double(), t[k]) <= 2e-2, n
        return
    r = oracle.reference_cpu_step(src, dst, V, X, *w, dY, agg, "leaky", 0.2)
    assert_parity(Y, r["Y"], t["Y"], 1e-5, "Y")
    assert_parity(dX, r["dX"], t["dX"], 1e-5, "dX")
    for p in parts:      # every rank holds the same all-reduced weight gradients
        for n, k in names.items():
            assert_parity(p["grads"][n], r[k], t[k], 1e-5, n)

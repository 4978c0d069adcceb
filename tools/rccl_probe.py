#!/usr/bin/env python3
"""RCCL check of the edge-cut layer: N ranks (torch.distributed.run), backend nccl (= RCCL), the
real native edge kernels and the async sparse halo all-to-all (sirgcn.dist); rank 0 checks the
assembled output and gradients against the single-GPU layer.  Needs one GPU per rank: RCCL
rejects two ranks on one device (ncclCommInitRank "invalid usage", measured on the 1-GPU builder
box, tools/gpu/r02c_rccl.sh), so on a 1-GPU box it cannot run; each rank uses cuda:LOCAL_RANK.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/rccl_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch import nn  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    from sirgcn import Graph, SIRConv
    from sirgcn.dist import DistGraph, DistSIRConv
    from sirgcn.synth import powerlaw_edges
    V, E, H = 20000, 400000, 256
    src, dst = powerlaw_edges(V, E, 0.8, seed=5)
    X = torch.randn(V, H, generator=torch.Generator().manual_seed(1)).to(dev)
    dY = torch.randn(V, H, generator=torch.Generator().manual_seed(2)).to(dev)
    ok = True
    for agg in ("sum", "sym", "mean"):
        torch.manual_seed(3)
        conv = SIRConv(H, H, H, nn.LeakyReLU(0.2), 0, agg_type=agg).to(dev)
        dg = DistGraph.from_global(src, dst, V, rank, world, dev)
        dconv = DistSIRConv(conv)
        r0, r1 = dg.row_begin, dg.row_end
        Xl = X[r0:r1].clone().requires_grad_(True)
        Y = dconv(dg, Xl)
        Y.backward(dY[r0:r1])
        dconv.allreduce_grads()
        torch.cuda.synchronize()
        # gather the row blocks on rank 0
        Ys = [torch.empty(0)] * world
        parts = {"Y": Y.detach(), "dX": Xl.grad.detach()}
        gathered = {}
        for k, t in parts.items():
            rows = torch.tensor([t.shape[0]], device=dev)
            allr = [torch.zeros_like(rows) for _ in range(world)]
            dist.all_gather(allr, rows)
            mx = int(max(int(r.item()) for r in allr))
            pad = torch.zeros(mx, t.shape[1], device=dev, dtype=t.dtype)
            pad[: t.shape[0]] = t
            bufs = [torch.zeros_like(pad) for _ in range(world)]
            dist.all_gather(bufs, pad)
            gathered[k] = torch.cat([b[: int(r.item())] for b, r in zip(bufs, allr)])
        grads = {n: p.grad.detach().clone() for n, p in conv.named_parameters()}
        if rank == 0:
            conv.zero_grad(set_to_none=True)
            x1 = X.clone().requires_grad_(True)
            Y1 = conv(Graph(src, dst, V), x1)
            Y1.backward(dY)
            ref = {"Y": Y1.detach(), "dX": x1.grad}
            ref.update({n: p.grad for n, p in conv.named_parameters()})
            got = dict(gathered)
            got.update(grads)
            for k in ref:
                e = ((got[k].double() - ref[k].double()).norm() / ref[k].double().norm().clamp_min(1e-30)).item()
                flag = e < 1e-5
                ok &= flag
                print(f"[rccl_probe] world={world} agg={agg} {k}: rel err {e:.2e} {'ok' if flag else 'FAIL'}", flush=True)
        dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        print("[rccl_probe]", "PASS" if ok else "FAIL", flush=True)
        sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

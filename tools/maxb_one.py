#!/usr/bin/env python3
"""One S1-shaped max layer (V=500k, E=10M, H=O=256, LeakyReLU 0.2): forward once, then the routed max
backward `--reps` times (for rocprofv3 --pmc passes over the backward kernels alone), plus the graph's
degree statistics (rows by degree, entries per arg edge)."""
import argparse
import sys
import os

import torch
from torch import nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sir-gcn_amd"))
from sirgcn import SIRConv, _native, edgemlp           # noqa: E402
from sirgcn.graph import get_plan                      # noqa: E402
from sirgcn.synth import powerlaw_graph                # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--V", type=int, default=500_000)
    ap.add_argument("--E", type=int, default=10_000_000)
    ap.add_argument("--H", type=int, default=256)
    a = ap.parse_args()
    _native.load()
    dev = torch.device("cuda")
    g = powerlaw_graph(a.V, a.E, 0.8, seed=0)
    plan = get_plan(g, dev)
    torch.manual_seed(0)
    m = SIRConv(a.H, a.H, a.H, nn.LeakyReLU(0.2), 0, agg_type="max").to(dev)
    X = torch.randn(a.V, a.H, device=dev)
    with torch.no_grad():
        QK = m._project(X, X) if hasattr(m, "_project") else None
    Q, K = QK[:, :a.H].contiguous(), QK[:, a.H:].contiguous()
    W, b = m.linear_relation.weight.detach().contiguous(), m.linear_relation.bias.detach().contiguous()
    Y = torch.empty(a.V, a.H, device=dev)
    arg = torch.empty(a.V, a.H, device=dev, dtype=torch.int32)
    edgemlp._fwd(plan, Q, K, W, b, "max", _native.ACT_LEAKY, 0.2, _native.ACT_IDENTITY, Y, arg)
    dY = torch.randn(a.V, a.H, device=dev)
    deg = (plan.dst.rowptr[1:] - plan.dst.rowptr[:-1]).long()
    sdeg = (plan.src.rowptr[1:] - plan.src.rowptr[:-1]).long()
    for name, d in (("dst", deg), ("src", sdeg)):
        q = torch.quantile(d.float(), torch.tensor([0.1, 0.25, 0.5, 0.75, 0.9, 0.99], device=dev)).tolist()
        print(f"{name} degree: max {int(d.max())} mean {float(d.float().mean()):.1f} quantiles(10/25/50/75/90/99) "
              f"{[round(x, 1) for x in q]}; rows deg<=8: {float((d <= 8).float().mean()):.3f}; "
              f"items {plan.dst.n_items if name == 'dst' else plan.src.n_items}")
    dQ, dK = torch.empty_like(Q), torch.empty_like(K)
    for _ in range(a.reps):
        edgemlp._max_bwd_sparse(plan, Q, K, W, arg, dY, _native.ACT_LEAKY, 0.2, dQ, dK)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Routed vs edge-materialised max backward on a small random graph: relative error per output
(dQ, dK, dW, db) — which kernel of the routed backward disagrees."""
import os
import sys

import torch
from torch import nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "sir-gcn_amd"))
from sirgcn import SIRConv, _native, edgemlp            # noqa: E402
from sirgcn.graph import Graph, get_plan                # noqa: E402

_native.load()
dev = torch.device("cuda")
for (V, E, H, O, chunk) in ((300, 3000, 128, 96, 256), (2000, 40000, 256, 256, 256)):
    gen = torch.Generator().manual_seed(1)
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V - 25, (E,), generator=gen)
    dst[:500] = 7
    g = Graph(src, dst, V)
    plan = get_plan(g, dev, chunk)
    Q = torch.randn(V, H, generator=gen).to(dev)
    K = torch.randn(V, H, generator=gen).to(dev)
    W = torch.randn(O, H, generator=gen).to(dev) * 0.1
    b = torch.randn(O, generator=gen).to(dev)
    Y = torch.empty(V, O, device=dev)
    arg = torch.empty(V, O, device=dev, dtype=torch.int32)
    edgemlp._fwd(plan, Q, K, W, b, "max", _native.ACT_LEAKY, 0.2, _native.ACT_IDENTITY, Y, arg)
    dY = torch.randn(V, O, generator=gen).to(dev)
    dQa, dKa = torch.empty_like(Q), torch.empty_like(K)
    dQb, dKb = torch.empty_like(Q), torch.empty_like(K)
    wa, ba = edgemlp._max_bwd_sparse(plan, Q, K, W, arg, dY, _native.ACT_LEAKY, 0.2, dQa, dKa)
    wb, bb = edgemlp._max_bwd_materialised(plan.dst, plan.src, Q, K, W, arg, dY, _native.ACT_LEAKY, 0.2, dQb, dKb)
    torch.cuda.synchronize()
    def rel(x, y):
        return float((x - y).norm() / y.norm().clamp_min(1e-30))
    print(os.environ.get("SIR_MAXB_DBG"), f"V{V} E{E} H{H} O{O} c{chunk}: dQ {rel(dQa, dQb):.2e} dK {rel(dKa, dKb):.2e} dW {rel(wa, wb):.2e} "
          f"db {rel(ba, bb):.2e}")
    bad = ((dQa - dQb).abs() > 1e-3 * dQb.abs().max()).any(1).nonzero().flatten()[:10].tolist()
    print("   first bad dQ rows", bad)

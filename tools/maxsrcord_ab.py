#!/usr/bin/env python3
"""A/B of the max layer's default (hybrid) backward under an env switch (--env) read by the library per call
(round 6 used it for SIR_MAXB_SRCORD — the dK pass on source-ordered entries — and SIR_MAXB_SPLIT — each
edge's entries over both half-waves; both measured slower and removed, profiles/r06_ab_maxb_*.txt), on an S1-shaped max layer
(V=500k, E=10M, H=O=256, LeakyReLU 0.2), interleaved in one process; dQK, dW_R, db_R compared
with the first form (bit-identical, or the largest relative L2 difference).  Times the whole backward (routing table, reorder, dQ / dK passes, dW_R)."""
import argparse
import os
import statistics
import sys

import torch
from torch import nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sir-gcn_amd"))
from sirgcn import SIRConv, _native                    # noqa: E402
from sirgcn.edgemlp import EdgeMaxLinear               # noqa: E402
from sirgcn.graph import get_plan                      # noqa: E402
from sirgcn.synth import powerlaw_graph                # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--V", type=int, default=500_000)
    ap.add_argument("--E", type=int, default=10_000_000)
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--forms", default="0,1")
    ap.add_argument("--env", default="SIR_MAXB_SRCORD")
    a = ap.parse_args()
    _native.load()
    dev = torch.device("cuda")
    g = powerlaw_graph(a.V, a.E, 0.8, seed=0)
    plan = get_plan(g, dev)
    torch.manual_seed(0)
    m = SIRConv(a.H, a.H, a.H, nn.LeakyReLU(0.2), 0, agg_type="max").to(dev)
    X = torch.randn(a.V, a.H, device=dev)
    with torch.no_grad():
        QK0 = m._project(X, X)
    W, b = m.linear_relation.weight, m.linear_relation.bias
    dY = torch.randn(a.V, a.H, device=dev)
    forms = a.forms.split(",")
    outs, times = {}, {f: [] for f in forms}
    for r in range(a.rounds):
        for f in forms:
            os.environ[a.env] = f
            QK = QK0.clone().requires_grad_(True)
            W.grad = b.grad = None
            Y = EdgeMaxLinear.apply(QK, W, b, plan, a.H, _native.ACT_LEAKY, 0.2)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            Y.backward(dY)
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[f].append(e0.elapsed_time(e1))
            outs[f] = (QK.grad.clone(), W.grad.clone(), b.grad.clone())
    for f in forms:
        same = all(torch.equal(x, y) for x, y in zip(outs[f], outs[forms[0]]))
        rel = max(float((x - y).norm() / y.norm().clamp_min(1e-30)) for x, y in zip(outs[f], outs[forms[0]]))
        print(f"{a.env}={f}: backward {statistics.median(times[f]):.3f} ms (min {min(times[f]):.3f}), "
              f"bit-identical to {forms[0]}: {same} (max relL2 {rel:.2e})", flush=True)


if __name__ == "__main__":
    main()

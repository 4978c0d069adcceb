#!/usr/bin/env python3
"""A/B of the max layer's default (hybrid) backward between library builds (same C ABI), interleaved in
one process, on an S1-shaped max layer (V=500k, E=10M, H=O=256, LeakyReLU 0.2; --graph S2 for the S2
shape); dQK, dW_R, db_R must be bit-identical.  Times the whole backward (routing table, dQ / dK passes,
dW_R).
    python tools/maxbwd_ab.py --libs new=sir-gcn_amd/lib/libsirconv.so old=/path/to/old.so"""
import argparse
import ctypes
import os
import statistics
import sys

import torch
from torch import nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sir-gcn_amd"))
from sirgcn import SIRConv, _native                    # noqa: E402
from sirgcn.edgemlp import EdgeMaxLinear               # noqa: E402
from sirgcn.graph import get_plan                      # noqa: E402
from sirgcn.synth import NAMED, powerlaw_graph         # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--graph", default="S1")
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--libs", nargs="+", required=True)
    a = ap.parse_args()
    _native.load()
    dev = torch.device("cuda")
    V, E, alpha = NAMED[a.graph]
    g = powerlaw_graph(V, E, alpha, seed=0)
    plan = get_plan(g, dev)
    torch.manual_seed(0)
    m = SIRConv(a.H, a.H, a.H, nn.LeakyReLU(0.2), 0, agg_type="max").to(dev)
    X = torch.randn(V, a.H, device=dev)
    with torch.no_grad():
        QK0 = m._project(X, X)
    W, b = m.linear_relation.weight, m.linear_relation.bias
    dY = torch.randn(V, a.H, device=dev)
    libs = []
    for kv in a.libs:
        name, path = kv.split("=", 1)
        h = ctypes.CDLL(path)
        for fn, (res, args) in _native.SIGNATURES.items():
            f = getattr(h, fn, None)
            if f is not None:
                f.restype, f.argtypes = res, args
        libs.append((name, h))
    outs, times = {}, {n: [] for n, _ in libs}
    for r in range(a.rounds):
        for n, h in libs:
            _native._lib = h
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
                times[n].append(e0.elapsed_time(e1))
            outs[n] = (QK.grad.clone(), W.grad.clone(), b.grad.clone())
    base = libs[0][0]
    for n, _ in libs:
        same = all(torch.equal(x, y) for x, y in zip(outs[n], outs[base]))
        print(f"{a.graph} {n}: backward {statistics.median(times[n]):.3f} ms (min {min(times[n]):.3f}), "
              f"bit-identical to {base}: {same}", flush=True)


if __name__ == "__main__":
    main()

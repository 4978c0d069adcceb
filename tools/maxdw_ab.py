#!/usr/bin/env python3
"""A/B of the max backward's dW_R / db_R kernels (sir_max_dw_qk: SIR_MAXDW=1 k_max_dw_qk, 4-row / 64-edge
batches; 2 k_max_dw_qk2, 16-row / 128-edge batches) on an S1-shaped max layer (V=500k, E=10M, H=O=256,
LeakyReLU 0.2), interleaved in one process; the outputs must be bit-identical."""
import argparse
import ctypes
import os
import statistics
import sys

import torch
from torch import nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sir-gcn_amd"))
from sirgcn import SIRConv, _native, edgemlp           # noqa: E402
from sirgcn.graph import get_plan                      # noqa: E402
from sirgcn.synth import powerlaw_graph                # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--V", type=int, default=500_000)
    ap.add_argument("--E", type=int, default=10_000_000)
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--forms", default="1,2", help="SIR_MAXDW values, each optionally @<lib name>")
    ap.add_argument("--libs", nargs="*", default=[], help="name=path of A/B library builds (same ABI)")
    a = ap.parse_args()
    _native.load()
    dev = torch.device("cuda")
    g = powerlaw_graph(a.V, a.E, 0.8, seed=0)
    plan = get_plan(g, dev)
    torch.manual_seed(0)
    m = SIRConv(a.H, a.H, a.H, nn.LeakyReLU(0.2), 0, agg_type="max").to(dev)
    X = torch.randn(a.V, a.H, device=dev)
    with torch.no_grad():
        QK = m._project(X, X)
    Q, K = QK[:, :a.H].contiguous(), QK[:, a.H:].contiguous()
    W, b = m.linear_relation.weight.detach().contiguous(), m.linear_relation.bias.detach().contiguous()
    Y = torch.empty(a.V, a.H, device=dev)
    arg = torch.empty(a.V, a.H, device=dev, dtype=torch.int32)
    edgemlp._fwd(plan, Q, K, W, b, "max", _native.ACT_LEAKY, 0.2, _native.ACT_IDENTITY, Y, arg)
    dY = torch.randn(a.V, a.H, device=dev)
    forms = a.forms.split(",")
    libs = {"main": _native.load()}
    for kv in a.libs:
        name, path = kv.split("=", 1)
        h = ctypes.CDLL(path)
        for fn, (res, args) in _native.SIGNATURES.items():
            f = getattr(h, fn, None)
            if f is not None:
                f.restype, f.argtypes = res, args
        libs[name] = h
    outs, times = {}, {f: [] for f in forms}
    for r in range(a.rounds):
        for f in forms:
            form, _, lib = f.partition("@")
            os.environ["SIR_MAXDW"] = form
            _native._lib = libs[lib or "main"]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dW, db = _native.max_dw_qk(plan.dst, arg, dY, Q, K, a.H, _native.ACT_LEAKY, 0.2)
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[f].append(e0.elapsed_time(e1))
            outs[f] = (dW, db)
    for f in forms:
        same = torch.equal(outs[f][0], outs[forms[0]][0]) and torch.equal(outs[f][1], outs[forms[0]][1])
        print(f"SIR_MAXDW={f}: {statistics.median(times[f]):.3f} ms (min {min(times[f]):.3f}), "
              f"bit-identical to {forms[0]}: {same}", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""A/B of the max layer's fused forward (sir_edge_mlp_fwd_stream at H = 256; fp32 split-fp16 form, or
the 16-bit form with --dtype bf16 / f16) between library builds (same C ABI), interleaved in one process,
on an S1-shaped layer (V=500k, E=10M, H=O=256, LeakyReLU 0.2); Y and the arg edges must be bit-identical.
    python tools/mlpfwd_ab.py --libs base=sir-gcn_amd/lib/libsirconv.so swz0=sir-gcn_amd/lib/libsirconv_swz0.so"""
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
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16", "f16"])
    ap.add_argument("--libs", nargs="+", required=True, help="name=path of library builds (same ABI)")
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
    dt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    QK = QK.to(dt)
    Q, K = QK[:, :a.H], QK[:, a.H:]
    W, b = m.linear_relation.weight.detach().contiguous(), m.linear_relation.bias.detach().contiguous()
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
            Y = torch.empty(a.V, a.H, device=dev)
            arg = torch.empty(a.V, a.H, device=dev, dtype=torch.int32)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if dt == torch.float32:
                edgemlp._fwd(plan, Q, K, W, b, "max", _native.ACT_LEAKY, 0.2, _native.ACT_IDENTITY, Y, arg)
            else:
                edgemlp._fwd_st(plan, Q, K, W, b, _native.ACT_LEAKY, 0.2, Y, arg)
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[n].append(e0.elapsed_time(e1))
            outs[n] = (Y, arg)
    base = libs[0][0]
    for n, _ in libs:
        same = torch.equal(outs[n][0], outs[base][0]) and torch.equal(outs[n][1], outs[base][1])
        print(f"{a.dtype} {n}: {statistics.median(times[n]):.3f} ms (min {min(times[n]):.3f}), "
              f"bit-identical to {base}: {same}", flush=True)


if __name__ == "__main__":
    main()

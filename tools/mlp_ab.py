#!/usr/bin/env python3
"""A/B the fused per-edge dense layer forward (sir_edge_mlp_fwd: agg='max' with W_R, or the
Sequential sigma's sum) of several builds of libsirconv, interleaved in ONE process, on a named
graph; checks every build's output (and max arg) is bit-identical to the first.

    make -C sir-gcn_amd/csrc VARIANT=mlpold DEFS=-DSIR_MLP_PIPE=0
    python tools/mlp_ab.py --graph S1 --libs new=sir-gcn_amd/lib/libsirconv.so old=sir-gcn_amd/lib/libsirconv_mlpold.so
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from gemm_ab import open_lib  # noqa: E402
from sirgcn import _native  # noqa: E402
from sirgcn.graph import get_plan  # noqa: E402
from sirgcn.synth import NAMED, molecule_batch, powerlaw_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="S1")
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--F", type=int, default=256)
    ap.add_argument("--agg", default="max", choices=["max", "sum", "mean", "sym"])
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--libs", nargs="+", required=True)
    a = ap.parse_args()
    dev = "cuda"
    if a.graph == "mol":
        g = molecule_batch(128, 23, seed=0)
    else:
        V, E, al = NAMED[a.graph]
        g = powerlaw_graph(V, E, al, seed=0)
    plan = get_plan(g, torch.device(dev))
    csr = plan.dst
    V = csr.n_rows
    gen = torch.Generator(device=dev).manual_seed(1)
    QK = torch.randn(V, 2 * a.H, device=dev, generator=gen)
    W = torch.randn(a.F, a.H, device=dev, generator=gen) / a.H ** 0.5
    b = torch.randn(a.F, device=dev, generator=gen)
    Q, K = QK[:, :a.H], QK[:, a.H:]
    in_norm, out_norm = plan.norms(a.agg if a.agg != "max" else "sum")
    code = 3 if a.agg == "max" else _native.AGG[a.agg]
    act2 = _native.ACT_IDENTITY if a.agg == "max" else _native.ACT_RELU
    P = _native._ptr
    st = _native._stream(torch.device(dev))
    libs, stream = [], {}
    for kv in a.libs:
        name, path = kv.split("=", 1)
        path, _, mode = path.partition("@")        # name=path@stream: the edge-stream entry point
        libs.append((name, open_lib(path)))
        stream[name] = mode == "stream"
    from sirgcn.edgemlp import _edge_rows
    erow = _edge_rows(csr)
    n = csr.n_slots
    pval = torch.empty((max(n, 1) * a.F,), device=dev)
    parg = torch.empty((max(n, 1) * a.F,), device=dev, dtype=torch.int32)
    outs, packs, works = {}, {}, {}
    for name, lib in libs:
        pk = torch.empty((lib.sir_edge_mlp_pack_bytes(a.H, a.F),), dtype=torch.uint8, device=dev)
        assert lib.sir_edge_mlp_pack(P(W), a.H, a.F, P(pk), st) == 0
        packs[name] = pk
        outs[name] = (torch.empty(V, a.F, device=dev), torch.empty(V, a.F, device=dev, dtype=torch.int32))
        if stream[name]:
            works[name] = torch.empty((lib.sir_edge_mlp_stream_work_bytes(a.F),), dtype=torch.uint8, device=dev)

    def run(name, lib):
        Y, arg = outs[name]
        if stream[name]:
            work = works[name]
            rc = lib.sir_edge_mlp_fwd_stream(P(csr.rowptr), P(csr.col), P(erow), csr.n_rows, csr.col.numel(), a.H, a.F,
                                             P(Q), Q.stride(0), P(K), K.stride(0), P(in_norm), P(out_norm), code,
                                             _native.ACT_LEAKY, 0.2, act2, P(packs[name]), P(b), P(Y), Y.stride(0),
                                             P(arg) if a.agg == "max" else None, a.F, P(work), st)
            assert rc == 0, lib.sir_last_error()
            return
        rc = lib.sir_edge_mlp_fwd(P(csr.rowptr), P(csr.col), P(csr.items), csr.n_items, P(csr.splits), csr.n_splits,
                                  a.H, a.F, P(Q), Q.stride(0), P(K), K.stride(0), P(in_norm), P(out_norm), code,
                                  _native.ACT_LEAKY, 0.2, act2, P(packs[name]), P(b), P(Y), Y.stride(0),
                                  P(arg) if a.agg == "max" else None, a.F, P(pval), P(parg) if a.agg == "max" else None,
                                  st)
        assert rc == 0, lib.sir_last_error()

    times = {name: [] for name, _ in libs}
    for _ in range(a.rounds):
        for name, lib in libs:
            run(name, lib)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(name, lib)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1))
    base = libs[0][0]
    E = csr.col.numel()
    for name, _ in libs:
        t = statistics.median(times[name])
        same = torch.equal(outs[name][0], outs[base][0]) and (a.agg != "max" or torch.equal(outs[name][1], outs[base][1]))
        rel = ((outs[name][0] - outs[base][0]).norm() / outs[base][0].norm()).item()
        print(f"{a.graph} {a.agg} H{a.H} F{a.F} {name:8s} {t:8.3f} ms (min {min(times[name]):8.3f})  "
              f"{2 * E * a.H * a.F / t / 1e9:7.1f} TFLOP/s fp32-equiv  bit-identical to {base}: {same} (relL2 {rel:.1e})", flush=True)


if __name__ == "__main__":
    main()

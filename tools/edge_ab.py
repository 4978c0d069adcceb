#!/usr/bin/env python3
"""A/B the edge passes of several builds of libsirconv (same C ABI, different compile flags) on
identical data, interleaved in ONE process (cdna_hip_programming.md §5.4 rule 24).

    make -C sir-gcn_amd/csrc VARIANT=nt DEFS=-DSIR_NT_STREAM=1
    python tools/edge_ab.py --graph S2 --libs base=sir-gcn_amd/lib/libsirconv.so nt=sir-gcn_amd/lib/libsirconv_nt.so
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))

import torch  # noqa: E402

from sirgcn import _native  # noqa: E402
from sirgcn.graph import GraphPlan  # noqa: E402
from sirgcn.synth import NAMED, powerlaw_edges  # noqa: E402


def open_lib(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _native.SIGNATURES.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="S2")
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--agg", default="sum")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16", "f16"])
    a = ap.parse_args()
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    dcode = _native.STORAGE[tdt]
    if a.graph == "mol":             # config 2's ZINC-shaped batch of 10,000 molecules (~2 in-edges per row)
        from sirgcn.synth import molecule_batch
        g0 = molecule_batch(10_000, 23, seed=0)
        src, dst = g0.edges()
        V, E = g0.num_nodes(), int(src.numel())
    else:
        V, E, alpha = NAMED[a.graph]
        src, dst = powerlaw_edges(V, E, alpha, seed=0)
    dev = "cuda"
    plan = GraphPlan(src, dst, V, dev, chunk=a.chunk)
    H = a.H
    g = torch.Generator(device=dev).manual_seed(0)
    QK = torch.randn(V, 2 * H, device=dev, generator=g).to(tdt)
    G = torch.randn(V, H, device=dev, generator=g).to(tdt)
    in_norm, out_norm = plan.norms(a.agg)
    nw = _native.mask_words(H, _native.ACT_LEAKY)
    mask = torch.empty(E * nw, device=dev, dtype=torch.int64)
    n_slots = max(plan.dst.n_slots, plan.src.n_slots)
    partial = torch.empty(max(n_slots, 1) * H, device=dev)
    outs = {}
    libs = [(kv.split("=", 1)[0], open_lib(kv.split("=", 1)[1])) for kv in a.libs]
    PASSES = ("fwd", "dst", "src", "both")
    times = {(n, p): [] for n, _ in libs for p in PASSES}
    partial_s = torch.empty(max(n_slots, 1) * H, device=dev)
    st = torch.cuda.current_stream()

    def run(lib):
        P = _native._ptr
        S = torch.empty(V, H, device=dev, dtype=tdt)
        dQK = torch.empty(V, 2 * H, device=dev, dtype=tdt)
        sp = ctypes.c_void_p(st.cuda_stream)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        d, s_ = plan.dst, plan.src
        Q, K = QK[:, :H], QK[:, H:]
        ev[0].record()
        rc = lib.sir_edge_agg_fwd(P(d.rowptr), P(d.col), P(d.items), d.n_items, P(d.splits), d.n_splits, H, dcode,
                                  P(Q), 2 * H, P(K), 2 * H, P(in_norm), P(out_norm), _native.AGG[a.agg],
                                  _native.ACT_LEAKY, 0.2, P(S), H, P(mask), P(partial), sp)
        ev[1].record()
        rc |= lib.sir_edge_agg_bwd_dst(P(d.rowptr), P(d.col), P(d.items), d.n_items, P(d.splits), d.n_splits, H, dcode,
                                       None, H, None, H, P(mask), P(G), H, P(in_norm), P(out_norm),
                                       _native.AGG[a.agg], _native.ACT_LEAKY, 0.2, P(dQK), 2 * H, None, H,
                                       P(partial), None, sp)
        ev[2].record()
        rc |= lib.sir_edge_agg_bwd_src(P(s_.rowptr), P(s_.col), P(s_.perm), P(s_.items), s_.n_items, P(s_.splits),
                                       s_.n_splits, H, dcode, None, H, None, H, P(mask), P(G), H, P(out_norm),
                                       P(in_norm), _native.AGG[a.agg], _native.ACT_LEAKY, 0.2,
                                       P(dQK[:, H:]), 2 * H, P(partial), None, sp)
        ev[3].record()
        # the one-launch backward (sum / sym): both passes again, into a second dQK
        dQK2 = torch.empty(V, 2 * H, device=dev, dtype=tdt)
        if a.agg in ("sum", "sym"):
            rc |= lib.sir_edge_agg_bwd(P(d.rowptr), P(d.col), P(d.items), d.n_items, P(d.splits), d.n_splits,
                                       P(s_.rowptr), P(s_.col), P(s_.perm), P(s_.items), s_.n_items, P(s_.splits),
                                       s_.n_splits, H, dcode, P(mask), P(G), H, P(in_norm), P(out_norm),
                                       _native.AGG[a.agg], _native.ACT_LEAKY, 0.2, P(dQK2), 2 * H, P(dQK2[:, H:]),
                                       2 * H, P(partial), P(partial_s), None, sp)
        ev[4].record()
        assert rc == 0, lib.sir_last_error()
        if a.agg in ("sum", "sym"):
            torch.cuda.synchronize()
            assert torch.equal(dQK2, dQK), "one-launch backward differs from the two passes"
        return ev, S, dQK

    for r in range(a.rounds):
        for name, lib in libs:
            ev, S, dQK = run(lib)
            torch.cuda.synchronize()
            if r == 0:
                outs[name] = (S, dQK)
            else:
                times[(name, "fwd")].append(ev[0].elapsed_time(ev[1]))
                times[(name, "dst")].append(ev[1].elapsed_time(ev[2]))
                times[(name, "src")].append(ev[2].elapsed_time(ev[3]))
                times[(name, "both")].append(ev[3].elapsed_time(ev[4]))
    base = libs[0][0]
    for name, _ in libs:
        same = torch.equal(outs[name][0], outs[base][0]) and torch.equal(outs[name][1], outs[base][1])
        med = {p: statistics.median(times[(name, p)]) for p in PASSES}
        mn = {p: min(times[(name, p)]) for p in PASSES}
        print(f"{name:10s} fwd {med['fwd']:.3f} ({mn['fwd']:.3f})  dst {med['dst']:.3f} ({mn['dst']:.3f})  "
              f"src {med['src']:.3f} ({mn['src']:.3f})  one-launch {med['both']:.3f} ({mn['both']:.3f}) ms   "
              f"bitwise-equal-to-{base}: {same}", flush=True)


if __name__ == "__main__":
    main()

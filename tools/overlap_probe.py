#!/usr/bin/env python3
"""Does a memory-bound edge pass overlap with independent fp32 GEMMs on a second stream?
Times (a) the dK (src) pass alone, (b) the GEMMs that do not depend on it alone, (c) both
issued on two streams.  S2 shapes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))
import torch  # noqa: E402

from sirgcn import _native  # noqa: E402
from sirgcn.conv import _tn  # noqa: E402
from sirgcn.graph import GraphPlan  # noqa: E402
from sirgcn.synth import NAMED, powerlaw_edges  # noqa: E402

V, E, alpha = NAMED[sys.argv[1] if len(sys.argv) > 1 else "S2"]
H = 256
dev = "cuda"
src, dst = powerlaw_edges(V, E, alpha, seed=0)
plan = GraphPlan(src, dst, V, dev)
g = torch.Generator(device=dev).manual_seed(0)
QK = torch.randn(V, 2 * H, device=dev, generator=g)
G = torch.randn(V, H, device=dev, generator=g)
X = torch.randn(V, H, device=dev, generator=g)
dY = torch.randn(V, H, device=dev, generator=g)
S = torch.randn(V, H, device=dev, generator=g)
W = torch.randn(2 * H, H, device=dev, generator=g)
nw = _native.mask_words(H, _native.ACT_LEAKY)
mask = torch.empty(E * nw, device=dev, dtype=torch.int64)
partial = torch.empty(max(plan.dst.n_slots, plan.src.n_slots, 1) * H, device=dev)
Sout = torch.empty(V, H, device=dev)
_native.edge_agg_fwd(plan.dst, QK[:, :H], QK[:, H:], None, None, "sum", _native.ACT_LEAKY, 0.2, Sout, partial, mask)
dQK = torch.empty(V, 2 * H, device=dev)
side = torch.cuda.Stream()


def edge():
    _native.edge_agg_bwd_src(plan.src, None, None, G, None, None, "sum", _native.ACT_LEAKY, 0.2, dQK[:, H:], partial, mask)


def gemms():
    _tn(dY, S)                       # dW_R
    torch.mm(dQK[:, :H], W[:H])      # dX (dQ part)
    _tn(dQK[:, :H].contiguous(), X)  # dW_Q


def both():
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        gemms()
    edge()
    cur.wait_stream(side)


def t(fn, n=5):
    fn(); torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for r in range(2):
    te, tg, tb = t(edge), t(gemms), t(both)
    print(f"edge {te:.3f} ms  gemms {tg:.3f} ms  sum {te + tg:.3f}  concurrent {tb:.3f} ms  saved {te + tg - tb:.3f}")

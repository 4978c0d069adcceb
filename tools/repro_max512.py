#!/usr/bin/env python3
"""Determinism / accuracy probe of the max form at H = O = 512 with hub rows split (chunk 64): the
layer run several times on the same inputs (dX must be bit-identical run to run), against the fp64
oracle; then with the QK projection on the native GEMMs (autograd nn.Linear on linalg) to see which
operand of dX = dQK W_cat differs.

    python tools/repro_max512.py"""
import os
import sys

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))
sys.path.insert(0, ROOT)
from sirgcn import Graph, SIRConv, linalg  # noqa: E402
from oracle import sirconv_oracle as oracle  # noqa: E402

DEV = "cuda"


def graph(seed, V=300, E=3000, dup=200):
    gen = torch.Generator().manual_seed(seed)
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V - 25, (E,), generator=gen)
    dst[:500] = 7
    idx = torch.randint(0, E, (dup,), generator=gen)
    return torch.cat([src, src[idx]]), torch.cat([dst, dst[idx]]), V, gen


def rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


def main():
    H = O = 512
    chunk = 64
    src, dst, V, gen = graph(H + O + chunk)
    d = 32
    X, dY = torch.randn(V, d, generator=gen), torch.randn(V, O, generator=gen)
    torch.manual_seed(O)
    m = SIRConv(d, H, O, nn.LeakyReLU(0.2), 0, agg_type="max").to(DEV)
    m.chunk = chunk
    g = Graph(src, dst, V)
    w = [t.detach().cpu().double() for t in (m.linear_query.weight, m.linear_query.bias, m.linear_key.weight,
                                              m.linear_relation.weight, m.linear_relation.bias)]
    r64 = oracle.reference_cpu_step(src, dst, V, X.double(), *w, dY.double(), "max", "leaky", 0.2)
    captured = {}

    def run():
        x = X.to(DEV).requires_grad_(True)
        m.zero_grad(set_to_none=True)
        orig = m._project

        def proj(fk, fq):
            QK = orig(fk, fq)
            QK.retain_grad()
            captured["QK"] = QK
            return QK
        m._project = proj
        try:
            Y = m(g, x)
            Y.backward(dY.to(DEV))
        finally:
            del m._project
        torch.cuda.synchronize()
        return Y.detach().cpu(), x.grad.cpu(), captured["QK"].grad.detach().cpu()

    outs = [run() for _ in range(6)]
    Wc = torch.cat([m.linear_query.weight, m.linear_key.weight], 0).detach().cpu().double()
    for i, (Y, dX, dQK) in enumerate(outs):
        print(f"run {i}: Y vs fp64 {rel(Y, r64['Y']):.2e}  dX vs fp64 {rel(dX, r64['dX']):.2e}  "
              f"dX vs dQK@W_cat(fp64) {rel(dX, dQK.double() @ Wc):.2e}  "
              f"dQK same as run 0: {torch.equal(dQK, outs[0][2])}  dX same as run 0: {torch.equal(dX, outs[0][1])}",
              flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Follow-up of tools/max_argflip.py (no arg flips: the native-route dX / dW_Q error of the H = O = 512
max case is not a near-tie): capture the layer's dQK and run the two GEMMs that consume it — dX = dQK W_cat
(mm_w) and [dW_Q; dW_K] = dQK^T X (mm_tn) — on each native route and on torch, against fp64; the operands
are saved to gpurun_out/max512_operands.pt for a CPU look.

    python tools/max_gemm_probe.py"""
import os
import sys

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))
sys.path.insert(0, ROOT)
from sirgcn import Graph, SIRConv, linalg, _native  # noqa: E402

DEV = "cuda"


def graph(seed, V=300, E=3000, dup=200):
    gen = torch.Generator().manual_seed(seed)
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V - 25, (E,), generator=gen)
    dst[:500] = 7
    idx = torch.randint(0, E, (dup,), generator=gen)
    return torch.cat([src, src[idx]]), torch.cat([dst, dst[idx]]), V, gen


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


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
    cap = {}
    orig = m._project

    def proj(fk, fq):
        QK = orig(fk, fq)
        QK.retain_grad()
        cap["QK"] = QK
        return QK
    m._project = proj
    x = X.to(DEV).requires_grad_(True)
    Y = m(g, x)
    Y.backward(dY.to(DEV))
    torch.cuda.synchronize()
    dQK = cap["QK"].grad.detach().contiguous()
    Wc = torch.cat([m.linear_query.weight, m.linear_key.weight], 0).detach().contiguous()
    Xd = X.to(DEV)
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save({"dQK": dQK.cpu(), "W_cat": Wc.cpu(), "X": X}, "gpurun_out/max512_operands.pt")
    ref_dx = dQK.double() @ Wc.double()
    ref_dw = dQK.double().t() @ Xd.double()
    a = dQK.abs()
    print(f"dQK: shape {tuple(dQK.shape)}, zeros {(dQK == 0).float().mean():.3f}, row max range "
          f"{a.max(1).values.min():.3e}..{a.max(1).values.max():.3e}, nonfinite {(~torch.isfinite(dQK)).sum().item()}")
    print(f"dX : direct {rel(_native.gemm_nt_direct(dQK, Wc, True), ref_dx):.2e}  packed "
          f"{rel(_native.gemm_nt(dQK, _native.gemm_pack(Wc, trans=True)), ref_dx):.2e}  torch "
          f"{rel(dQK @ Wc, ref_dx):.2e}")
    print(f"dW : native tn {rel(_native.gemm_tn(dQK, Xd), ref_dw):.2e}  torch {rel(dQK.t() @ Xd, ref_dw):.2e}")
    cs = _native.gemm_tn(dQK, Xd, colsum=True)
    print(f"dW (colsum) {rel(cs[0], ref_dw):.2e}  colsum {rel(cs[1], dQK.double().sum(0)):.2e}")
    # sigma' sign flips: z = Q[v] + K[u] from the GPU's fp32 QK vs from an fp64 projection
    import oracle
    QK32 = cap["QK"].detach().double().cpu()
    Wq, bq, Wk = (t.detach().cpu().double() for t in (m.linear_query.weight, m.linear_query.bias, m.linear_key.weight))
    Q64 = X.double() @ Wq.t() + bq
    K64 = X.double() @ Wk.t()
    z32 = QK32[dst, :H] + QK32[src, H:]
    z64 = Q64[dst] + K64[src]
    flip = (z32 > 0) != (z64 > 0)
    mag = (X.double().abs() @ Wq.abs().t() + bq.abs())[dst] + (X.double().abs() @ Wk.abs().t())[src]
    print(f"sigma' sign flips: {int(flip.sum())} of {flip.numel()}; their |z64| / (2^-24 mag): "
          f"{(z64[flip].abs() / (mag[flip] * 2.0 ** -24)).tolist()[:8]}")
    print(f"QK vs fp64 projection: {rel(QK32, torch.cat([Q64, K64], 1)):.2e}")
    # dQK scored against fp64 with the GPU's own QK (signs and arg as the kernel saw them)
    w = [t.detach().cpu().double() for t in (m.linear_query.weight, m.linear_query.bias, m.linear_key.weight,
                                             m.linear_relation.weight, m.linear_relation.bias)]
    r64 = oracle.reference_cpu_step(src, dst, V, X.double(), *w, dY.double(), "max", "leaky", 0.2)
    print(f"layer dX vs fp64 {rel(x.grad.cpu(), r64['dX']):.2e}")
    # per-row / per-column error localisation
    e = (_native.gemm_nt_direct(dQK, Wc, True).double() - ref_dx).norm(dim=1) / ref_dx.norm(dim=1).clamp_min(1e-30)
    print("dX worst rows:", [(int(i), f"{e[i]:.2e}") for i in e.argsort(descending=True)[:6]])
    e2 = (_native.gemm_tn(dQK, Xd).double() - ref_dw).norm(dim=1) / ref_dw.norm(dim=1).clamp_min(1e-30)
    print("dW worst rows:", [(int(i), f"{e2[i]:.2e}") for i in e2.argsort(descending=True)[:6]])


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""A/B the 16-bit NT GEMM (sir_gemm_nt16) of several builds of libsirconv on the autocast layer's
S2 shapes, interleaved in ONE process: QK (fp32 X rounded on load + rounded copy, N = 2H), Y and
G (16-bit A, N = H), dX (16-bit A, K = 2H, fp32 out).  ms median (min); d = max relative
difference to the first library.

    make -C sir-gcn_amd/csrc VARIANT=ns4 DEFS="-DSIR_NT16_NS=4"
    python tools/gemm16_ab.py --libs base=sir-gcn_amd/lib/libsirconv.so ns4=sir-gcn_amd/lib/libsirconv_ns4.so
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


def open_lib(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _native.SIGNATURES.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=2_000_000)
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--tn", nargs="*", default=[], help="also time sir_gemm_tn16 at R,M,N (e.g. 229532,256,128)")
    ap.add_argument("--no-nt", action="store_true")
    a = ap.parse_args()
    V, H, dev, dt = a.V, a.H, "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(V, H, device=dev, generator=g)
    S = torch.randn(V, H, device=dev, generator=g).to(dt)
    dQK = torch.randn(V, 2 * H, device=dev, generator=g).to(dt)
    W2 = torch.randn(2 * H, H, device=dev, generator=g) * H ** -0.5
    W1 = torch.randn(H, H, device=dev, generator=g) * H ** -0.5
    b2 = torch.randn(2 * H, device=dev, generator=g).to(dt).float()
    libs = [(kv.split("=", 1)[0], open_lib(kv.split("=", 1)[1])) for kv in a.libs]
    P = _native._ptr
    BF, F32 = 1, 0
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def pack(lib, W, trans):
        N, K = (W.shape[1], W.shape[0]) if trans else W.shape
        pk = torch.empty((lib.sir_gemm_pack16_bytes(N, K),), dtype=torch.uint8, device=dev)
        assert lib.sir_gemm_pack16(P(W), W.stride(0), N, K, int(trans), BF, P(pk), st) == 0
        return pk

    def shapes(lib):
        p2, p1, p1t, p2t = pack(lib, W2, False), pack(lib, W1, False), pack(lib, W1, True), pack(lib, W2, True)
        QK = torch.empty(V, 2 * H, device=dev, dtype=dt)
        Xh = torch.empty(V, H, device=dev, dtype=dt)
        Y = torch.empty(V, H, device=dev, dtype=dt)
        G = torch.empty(V, H, device=dev, dtype=dt)
        dX = torch.empty(V, H, device=dev, dtype=torch.float32)
        return [
            ("QK x32 N=2H", lambda: lib.sir_gemm_nt16(P(X), H, F32, V, H, P(p2), 2 * H, BF, P(b2), P(QK), 2 * H, BF, P(Xh), H, None, st), QK),
            ("Y  N=H", lambda: lib.sir_gemm_nt16(P(S), H, BF, V, H, P(p1), H, BF, None, P(Y), H, BF, None, 0, None, st), Y),
            ("G  N=H (W^T)", lambda: lib.sir_gemm_nt16(P(S), H, BF, V, H, P(p1t), H, BF, None, P(G), H, BF, None, 0, None, st), G),
            ("dX K=2H f32", lambda: lib.sir_gemm_nt16(P(dQK), 2 * H, BF, V, 2 * H, P(p2t), H, BF, None, P(dX), H, F32, None, 0, None, st), dX),
        ]

    def tn_shapes(lib):
        out = []
        g.manual_seed(1)          # the same operands for every library
        for spec in a.tn:
            R, M, N = (int(x) for x in spec.split(","))
            At = torch.randn(R, M, device=dev, generator=g).to(dt)
            Bt = torch.randn(R, N, device=dev, generator=g).to(dt)
            C = torch.empty(M, N, device=dev)
            cs = torch.empty(M, device=dev)
            ws = torch.empty((max(lib.sir_gemm_tn_workspace(R, M, N), 4),), dtype=torch.uint8, device=dev)
            out.append((f"tn16 {R}x{M}x{N}", (lambda At=At, Bt=Bt, C=C, cs=cs, ws=ws, R=R, M=M, N=N:
                        lib.sir_gemm_tn16(P(At), M, P(Bt), N, R, M, N, BF, P(C), N, P(cs), P(ws), ws.numel(), st)), C))
        return out

    runs = {n: ([] if a.no_nt else shapes(lib)) + tn_shapes(lib) for n, lib in libs}
    times = {}
    for r in range(a.rounds):
        for n, _ in libs:
            for name, fn, out in runs[n]:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert fn() == 0
                e1.record()
                torch.cuda.synchronize()
                if r > 0:
                    times.setdefault((n, name), []).append(e0.elapsed_time(e1))
    base = libs[0][0]
    tot = {}
    for i, (name, _, _) in enumerate(runs[base]):
        line = f"{name:14s}"
        for n, _ in libs:
            t = times[(n, name)]
            out, ref = runs[n][i][2].float(), runs[base][i][2].float()
            d = ((out - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()
            line += f" | {n} {statistics.median(t):7.3f} ms (min {min(t):7.3f}, d {d:.1e})"
            tot[n] = tot.get(n, 0.0) + statistics.median(t)
        print(line, flush=True)
    print("total: " + "  ".join(f"{n} {v:.3f} ms" for n, v in tot.items()))


if __name__ == "__main__":
    main()

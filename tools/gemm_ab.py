#!/usr/bin/env python3
"""A/B the projection GEMMs of several builds of libsirconv (same C ABI, different compile
flags) on the layer's shapes, interleaved in ONE process (cdna_hip_programming.md §5.4 rule 24).

    make -C sir-gcn_amd/csrc VARIANT=nt2 DEFS=-DSIR_NT_CFG=2
    python tools/gemm_ab.py --libs base=sir-gcn_amd/lib/libsirconv.so nt2=sir-gcn_amd/lib/libsirconv_nt2.so
Prints ms (median over rounds) per shape and library, and checks the outputs agree (bitwise
equality is not expected across tilings; the relative difference is printed)."""
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
        f = getattr(lib, name, None)        # an older A/B build may lack newer entry points
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=2_000_000)
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--only", default=None, help="run only the shapes whose name starts with this")
    ap.add_argument("--reps", type=int, default=1, help="back-to-back calls per timed sample (small shapes)")
    ap.add_argument("--torch", action="store_true", help="add torch's fp32 GEMM (hipBLASLt) as a column")
    a = ap.parse_args()
    V, H = a.V, a.H
    dev = "cuda"
    P = _native._ptr
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(V, H, device=dev, generator=g)
    D2 = torch.randn(V, 2 * H, device=dev, generator=g)
    W2 = torch.randn(2 * H, H, device=dev, generator=g) / H ** 0.5
    WR = torch.randn(H, H, device=dev, generator=g) / H ** 0.5
    b2 = torch.randn(2 * H, device=dev, generator=g)
    # name=path[@VAR=value]: the variable is set in the environment around every call of that library
    # (kernel routes the library reads per call, e.g. SIR_NT_G=1)
    libs, envs = [], {}
    for kv in a.libs:
        name, rest = kv.split("=", 1)
        path, _, env = rest.partition("@")
        libs.append((name, open_lib(path)))
        envs[name] = tuple(env.split("=", 1)) if env else None
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    if a.torch:
        libs.append(("torch", None))
        envs["torch"] = None

    def pack(lib, W, trans):
        N, K = (W.shape[1], W.shape[0]) if trans else W.shape
        pk = torch.empty(lib.sir_gemm_pack_bytes(N, K), dtype=torch.uint8, device=dev)
        assert lib.sir_gemm_pack(P(W), W.stride(0), N, K, int(trans), P(pk), st) == 0
        return pk, N, K

    shapes = {
        "QK  nt K=H  N=2H": (X, W2, False, b2),
        "Y   nt K=H  N=H": (X, WR, False, None),
        "G   nt^T    N=H": (X, WR, True, None),
        "dX  nt^T K=2H N=H": (D2, W2, True, None),
        "dWR tn": (X, X),
        "dW  tn": (D2, X),
    }
    if a.only:
        pre = a.only.split(",")
        shapes = {k: v for k, v in shapes.items() if any(k.startswith(x) for x in pre)}
    packs = {(n, s): pack(lib, v[1], v[2]) for n, lib in libs if lib is not None for s, v in shapes.items()
             if len(v) == 4}
    outs = {}
    ws = torch.empty(max(lib.sir_gemm_tn_workspace(V, 2 * H, H) for _, lib in libs if lib is not None),
                     dtype=torch.uint8, device=dev)

    def run(n, lib, s):
        if envs[n]:
            os.environ[envs[n][0]] = envs[n][1]
        else:
            for e in {x[0] for x in envs.values() if x}:
                os.environ.pop(e, None)
        v = shapes[s]
        if lib is None:                      # torch (hipBLASLt)
            if len(v) == 4:
                A, W, trans, bias = v
                Wt = W if trans else W.t()
                outs[(n, s)] = torch.addmm(bias, A, Wt) if bias is not None else A @ Wt
            else:
                outs[(n, s)] = v[0].t() @ v[1]
            return
        if len(v) == 4:
            A, _, _, bias = v
            pk, N, K = packs[(n, s)]
            C = outs.setdefault((n, s), torch.empty(V, N, device=dev))
            rc = lib.sir_gemm_nt(P(A), A.stride(0), V, K, P(pk), N, P(bias), P(C), C.stride(0), None, st)
        else:
            A, B = v
            C = outs.setdefault((n, s), torch.empty(A.shape[1], B.shape[1], device=dev))
            rc = lib.sir_gemm_tn(P(A), A.stride(0), P(B), B.stride(0), V, A.shape[1], B.shape[1], P(C),
                                 C.stride(0), None, P(ws), ws.numel(), st)
        assert rc == 0, lib.sir_last_error()

    times = {(n, s): [] for n, _ in libs for s in shapes}
    for _ in range(a.rounds):
        for s in shapes:
            for n, lib in libs:
                run(n, lib, s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    run(n, lib, s)
                e1.record()
                torch.cuda.synchronize()
                times[(n, s)].append(e0.elapsed_time(e1) / a.reps)
    base = libs[0][0]
    for s in shapes:
        row = [f"{s:20s}"]
        for n, _ in libs:
            t = statistics.median(times[(n, s)])
            d = (outs[(n, s)] - outs[(base, s)]).norm() / outs[(base, s)].norm()
            row.append(f"{n} {t:7.3f} ms (min {min(times[(n, s)]):7.3f}, d {d:.1e})")
        print(" | ".join(row), flush=True)
    for n, _ in libs:
        print(f"total {n}: {sum(statistics.median(times[(n, s)]) for s in shapes):.3f} ms")


if __name__ == "__main__":
    main()

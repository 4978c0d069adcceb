#!/usr/bin/env python3
"""HBM floors of the projection GEMM shapes on this GPU: torch streaming kernels that move the same
bytes as each GEMM (no arithmetic worth the name), timed with HIP events.  A GEMM at its memory floor
runs as fast as these.

    python tools/stream_floor.py [--V 2000000] [--H 256]"""
import argparse

import torch


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=2_000_000)
    ap.add_argument("--H", type=int, default=256)
    a = ap.parse_args()
    V, H = a.V, a.H
    X = torch.randn(V, H, device="cuda")
    X2 = torch.randn(V, 2 * H, device="cuda")
    Y = torch.empty(V, H, device="cuda")
    Y2 = torch.empty(V, 2 * H, device="cuda")
    s = torch.empty(H, device="cuda")
    s2 = torch.empty(2 * H, device="cuda")
    cases = [
        ("read H, write H (Y, G floor)", lambda: torch.mul(X, 2.0, out=Y), 2 * V * H * 4),
        ("read H, write 2H (QK floor)", lambda: Y2.view(V, 2, H).copy_(X.unsqueeze(1).expand(V, 2, H)), 3 * V * H * 4),
        ("read 2H, write H (dX floor)", lambda: torch.add(X2[:, :H], X2[:, H:], out=Y), 3 * V * H * 4),
        ("read H (column sums)", lambda: torch.sum(X, 0, out=s), V * H * 4),
        ("read H + H (dW_R floor)", lambda: (torch.sum(X, 0, out=s), torch.sum(Y, 0, out=s)), 2 * V * H * 4),
        ("read 2H + H (dW_QK floor)", lambda: (torch.sum(X2, 0, out=s2), torch.sum(X, 0, out=s)), 3 * V * H * 4),
        ("copy 2H", lambda: Y2.copy_(X2), 4 * V * H * 4),
    ]
    for name, fn, nbytes in cases:
        t = timeit(fn)
        print(f"{name:32s} {t:7.3f} ms  {nbytes / t / 1e9:7.3f} TB/s  ({nbytes / 1e9:.2f} GB)")


if __name__ == "__main__":
    main()

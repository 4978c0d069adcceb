#!/usr/bin/env python3
"""Random-row gather rate of this GPU by row size: how fast can ANY kernel read E rows of R bytes
picked at random from a table larger than the caches?  torch kernels (index_select: gathered read +
sequential write; embedding_bag sum: gathered read, small output), timed with HIP events, beside a
sequential copy of the same bytes.  The edge passes gather 1 KiB rows (fp32, H = 256) or 512-B rows
(bf16 / fp16 storage); this separates the row size's own cost from the kernels'.

    python tools/gather_floor.py [--V 2000000] [--E 20000000]"""
import argparse

import torch
import torch.nn.functional as F


def timeit(fn, reps=7):
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
    ap.add_argument("--E", type=int, default=20_000_000)
    a = ap.parse_args()
    V, E = a.V, a.E
    g = torch.Generator(device="cuda").manual_seed(0)
    idx = torch.randint(0, V, (E,), device="cuda", generator=g)
    deg = 20
    offsets = torch.arange(0, E, deg, device="cuda")
    for dt, width in ((torch.float32, 256), (torch.float32, 128), (torch.bfloat16, 256), (torch.float32, 512),
                      (torch.float32, 64)):
        table = torch.randn(V, width, device="cuda", generator=g).to(dt)
        rb = width * table.element_size()
        out = torch.empty(E, width, device="cuda", dtype=dt)
        t_is = timeit(lambda: torch.index_select(table, 0, idx, out=out))
        t_eb = None
        try:
            t_eb = timeit(lambda: F.embedding_bag(idx, table, offsets, mode="sum"))
        except RuntimeError:
            pass
        src = torch.empty_like(out)
        t_cp = timeit(lambda: out.copy_(src))
        gb = E * rb / 1e9
        line = (f"{str(dt):15s} row {rb:5d} B | index_select {t_is:7.3f} ms: gathered read {gb / t_is:6.3f} TB/s "
                f"(+ write: {2 * gb / t_is:6.3f}) | seq copy {2 * gb / t_cp:6.3f} TB/s")
        if t_eb is not None:
            line += f" | embedding_bag sum {t_eb:7.3f} ms: {gb / t_eb:6.3f} TB/s"
        print(line, flush=True)
        del table, out, src


if __name__ == "__main__":
    main()

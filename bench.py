#!/usr/bin/env python3
"""bench.py — edges/sec of one SIRConv layer, forward + backward, d_hidden = 256, on MI355X.

Metric (BASELINE.json): "edges/sec SIRConv fwd+bwd, d_hidden=256, 1/2/4/8 MI355X".
Workload (default, BASELINE config 4 / SURVEY §8d): synthetic Chung-Lu power-law graph S2
(V = 2,000,000, E = 40,000,000, alpha = 0.8; `sirgcn.synth`), d_in = H = d_out = 256 fp32,
agg = sum, sigma = LeakyReLU(0.2); X ~ N(0,1) (seed 3), nn.Linear default init (seed 4),
dY ~ N(0,1) (seed 5).  One step = Y = SIRConv(g, X); Y.backward(dY)  (projections, edge
kernels, all weight/input gradients).  Graph plan (CSR build) is outside the timed region,
as DGL's cached CSC is.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--graph S2|S1|S1u|arxiv] [--agg sum]
  N > 1: launched by torch.distributed.run, one rank per GPU; dst-range edge-cut of the SAME
  graph (strong scaling) with a sparse RCCL all-to-all of halo K rows fwd and its transpose for dK bwd (sirgcn.dist).

Prints ONE JSON line (rank 0).  `roofline` is for the dominant edge kernel, timed live with
HIP events on the launching stream; `cpu_baseline` is the reference CPU dataflow restated in
oracle/ (DGL edge-UDF path: gathers + index_add, torch autograd), on a bounded sample.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch import nn  # noqa: E402

METRIC = "edges/sec SIRConv fwd+bwd, d_hidden=256, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
FP32_PEAK_TFLOPS = 157.3    # fp32 MFMA = vector peak (no xf32 on gfx950)
FP16_PEAK_FLOPS = 2.5e15    # dense fp16/bf16 MFMA (MI355X_MICROARCH.md; the 5 PF figure is 2:1 sparse)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--graph", default="S2")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--agg", default="sum", choices=["sum", "mean", "sym"])
    ap.add_argument("--chunk", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) for real runs; gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the edge-cut (sirgcn.dist) code path even at world size 1")
    ap.add_argument("--torch-gemm", action="store_true",
                    help="A/B only: projections on torch fp32 GEMMs instead of the native MFMA kernels")
    ap.add_argument("--pmc-file", default=None,
                    help="PMC traffic summary (tools/pmc_traffic.py); default profiles/pmc_traffic_<graph>.json")
    return ap.parse_args()


def edge_pass_bytes(name, V_rows, E, H, agg, masked, s=4, si=4):
    """Algorithmic HBM bytes of one launch of each edge pass.

    Recompute mode (any sigma): fwd gathers K[u]; dQ pass re-gathers K[u]; dK pass gathers Q[v]
    and G[v].  Sign-mask mode (ReLU family): fwd also writes H bits/edge; dQ pass reads only the
    mask; dK pass gathers G[v] + the edge's mask words (+ its permutation index).
    """
    mb = 8 * 4 * ((H + 255) // 256) if masked else 0           # mask bytes per edge
    sym_e = E * (si + 4) if agg == "sym" else 0                 # col + norm_col per edge when c_e needed
    sym_r = V_rows * 4 if agg == "sym" else 0
    if name == "sir_edge_agg_fwd":       # col + K[u] (+ mask write) per edge; Q read + S write + rowptr
        return E * (si + H * s + mb) + V_rows * (2 * H * s + si) + (E * 4 if agg == "sym" else 0) + sym_r
    if name == "sir_edge_agg_bwd_dst":
        mean = V_rows * H * s if agg == "mean" else 0           # Gm side output
        if masked:                       # mask per edge; G read + dQ write per row
            return E * mb + sym_e + V_rows * (2 * H * s + si) + sym_r + mean
        return E * (si + H * s) + V_rows * (3 * H * s + si) + (E * 4 if agg == "sym" else 0) + sym_r + mean
    if name == "sir_edge_agg_bwd_src":
        if masked:                       # col + perm + G[v] + mask per edge; dK write per row
            return E * (2 * si + H * s + mb) + V_rows * (H * s + si) + (E * 4 if agg == "sym" else 0) + sym_r
        return E * (si + 2 * H * s) + V_rows * (2 * H * s + si) + (E * 4 if agg == "sym" else 0) + sym_r
    raise KeyError(name)


def cpu_baseline(args, H):
    """Reference CPU dataflow (oracle.reference_cpu_step) on a bounded sample, rank 0 only."""
    import oracle
    from sirgcn.synth import powerlaw_edges
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    Vs, Es = 100_000, 2_000_000
    src, dst = powerlaw_edges(Vs, Es, 0.8, seed=0)
    g = torch.Generator().manual_seed(3)
    X = torch.randn(Vs, H, generator=g)
    torch.manual_seed(4)
    m = nn.ModuleList([nn.Linear(H, H), nn.Linear(H, H, bias=False), nn.Linear(H, H)])
    dY = torch.randn(Vs, H, generator=torch.Generator().manual_seed(5))
    w = [m[0].weight.data, m[0].bias.data, m[1].weight.data, m[2].weight.data, m[2].bias.data]
    oracle.reference_cpu_step(src, dst, Vs, X, *w, dY, args.agg, "leaky", 0.2)    # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        oracle.reference_cpu_step(src, dst, Vs, X, *w, dY, args.agg, "leaky", 0.2)
        n += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or n >= 20:
            break
    cpu_model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": Es * n / el, "unit": "edges/s", "cores": cores, "kind": "port",
            "sample": f"Chung-Lu alpha=0.8 V={Vs} E={Es} H={H} {args.agg} LeakyReLU(0.2), "
                      f"{n} fwd+bwd steps in {el:.1f}s (oracle.reference_cpu_step: DGL edge-UDF dataflow, torch CPU autograd)",
            "cpu_model": cpu_model}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))     # one rank per GPU (wraps only in rehearsals)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from sirgcn import SIRConv, _native, linalg
    if args.torch_gemm:
        linalg.USE_NATIVE = False
    from sirgcn.graph import DEFAULT_CHUNK
    from sirgcn.synth import NAMED, powerlaw_edges
    H = args.hidden
    V, E, alpha = NAMED[args.graph]
    src, dst = powerlaw_edges(V, E, alpha, seed=0)

    torch.manual_seed(4)
    conv = SIRConv(H, H, H, nn.LeakyReLU(0.2, inplace=True), 0, agg_type=args.agg).to(dev)
    if args.chunk:
        conv.chunk = args.chunk
    gen = torch.Generator().manual_seed(3)
    X_full = torch.randn(V, H, generator=gen)
    dY_full = torch.randn(V, H, generator=torch.Generator().manual_seed(5))

    dconv = None
    if world == 1 and not args.force_dist:
        from sirgcn import Graph
        g = Graph(src, dst, V)
        X = X_full.to(dev).requires_grad_(True)
        dY = dY_full.to(dev)
        layer = lambda: conv(g, X)
        rows_local, edges_local = V, E
        rows_src = V
    else:
        from sirgcn.dist import DistGraph, DistSIRConv
        dg = DistGraph.from_global(src, dst, V, rank, world, dev, chunk=args.chunk or DEFAULT_CHUNK)
        dconv = DistSIRConv(conv)
        r0, r1 = dg.row_begin, dg.row_end
        X = X_full[r0:r1].to(dev).requires_grad_(True)
        dY = dY_full[r0:r1].to(dev)
        layer = lambda: dconv(dg, X)
        rows_local, edges_local = r1 - r0, dg.num_local_edges
        rows_src = dg.n_ext
    del X_full, dY_full

    def step():
        conv.zero_grad(set_to_none=True)
        X.grad = None
        Y = layer()
        Y.backward(dY)
        if dconv is not None:
            dconv.allreduce_grads()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timing = _native.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    _native.enable_timing(False)
    el_t = torch.tensor([el], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = el_t.item()
    ms = 1e3 * el / args.steps

    from sirgcn.conv import EdgeAggregate
    masked = bool(EdgeAggregate.use_mask and _native.mask_words(H, _native.ACT_LEAKY))
    kernels, gemm = {}, {}
    for name, evs in timing.items():
        t = sum(a.elapsed_time(b) for a, b, _ in evs) / len(evs)    # ms per launch
        if name.startswith("sir_gemm_"):       # MFMA-bound projections: flops per launch
            if name == "sir_gemm_pack":
                continue
            fl = sum(w for _, _, w in evs) / len(evs)
            gemm[name] = {"ms": round(t, 4), "launches": len(evs), "flops": fl,
                          "TFLOPs": round(fl / (t * 1e-3) / 1e12, 1)}
            continue
        bytes_ = edge_pass_bytes(name, rows_local if name != "sir_edge_agg_bwd_src" else rows_src, edges_local, H,
                                 args.agg, masked)
        kernels[name] = {"ms": round(t, 4), "launches": len(evs), "bytes": bytes_,
                         "GBps": round(bytes_ / (t * 1e-3) / 1e9, 1)}
    dom = max(kernels, key=lambda k: kernels[k]["ms"])
    traffic = None
    pmc_file = args.pmc_file or os.path.join(ROOT, "profiles", f"pmc_traffic_{args.graph}.json")
    try:
        with open(pmc_file) as f:
            pmc = json.load(f)
        rec = pmc.get("kernels", {}).get(dom)
        if (rec and world == 1 and pmc.get("graph") == args.graph and pmc.get("agg") == args.agg
                and pmc.get("H") == H):
            traffic = rec["hbm_bytes_per_launch"]      # L2<->fabric bytes (Infinity-Cache hits included)
    except (OSError, ValueError):
        pass
    d = kernels[dom]
    roofline = {"bound": "hbm", "kernel": dom, "backward_mode": "sign-mask" if masked else "recompute", "achieved": d["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(d["GBps"] / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes": d["bytes"], "ms_per_launch": d["ms"], "all_kernels": kernels}

    out = {"metric": METRIC, "value": round(E / (el / args.steps), 1), "unit": "edges/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
           "config": {"workload": f"{args.graph}: Chung-Lu power-law V={V} E={E} alpha={alpha}; 1 SIRConv layer "
                                  f"d_in=H=d_out={H}, agg={args.agg}, LeakyReLU(0.2); fwd+bwd incl. projections",
                      "graph": args.graph, "V": V, "E": E, "hidden": H, "agg": args.agg,
                      "parallelism": f"edge-cut dst-range x{world}, sparse halo all-to-all" if world > 1
                      else "single GPU"},
           "roofline": roofline}
    if gemm:   # projections (split-fp16 MFMA): fp32-equivalent flops; raw fp16 MFMA work is 3x that
        fl = sum(g["flops"] * g["launches"] for g in gemm.values()) / args.steps
        tg = sum(g["ms"] * g["launches"] for g in gemm.values()) / args.steps
        out["projections"] = {"bound": "mfma", "ms_per_step": round(tg, 3), "flops_per_step": fl,
                              "achieved_fp32_equiv_TFLOPs": round(fl / (tg * 1e-3) / 1e12, 1),
                              "fp16_mfma_util": round(3 * fl / (tg * 1e-3) / FP16_PEAK_FLOPS, 4),
                              "vs_fp32_peak": round(fl / (tg * 1e-3) / (FP32_PEAK_TFLOPS * 1e12), 3),
                              "kernels": gemm}
    if dconv is not None:     # halo exchange volume per rank (rows of H fp32), max over ranks
        ex = torch.tensor([dg.n_halo, int(dg.send_idx.numel()), edges_local], dtype=torch.float64,
                          device=dev if args.dist_backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(ex, op=dist.ReduceOp.MAX)
        out["exchange"] = {"halo_rows_max": int(ex[0]), "send_rows_max": int(ex[1]), "local_edges_max": int(ex[2]),
                           "bytes_per_direction_max": int(ex[0]) * H * 4,
                           "dense_allgather_rows": V - min(dg.bounds[i + 1] - dg.bounds[i] for i in range(world))}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, H)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

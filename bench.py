#!/usr/bin/env python3
"""bench.py — edges/sec of SIRConv forward + backward on MI355X (BASELINE.json metric).

Default workload (BASELINE config 4 / SURVEY §8d): synthetic Chung-Lu power-law graph S2
(V = 2,000,000, E = 40,000,000, alpha = 0.8; ``sirgcn.synth``), ONE SIRConv layer,
d_in = H = d_out = 256, fp32, agg = sum, sigma = LeakyReLU(0.2); X ~ N(0,1) (seed 3),
nn.Linear default init (seed 4), dY ~ N(0,1) (seed 5).  One step = Y = SIRConv(g, X);
Y.backward(dY) (projections, edge kernels, every weight / input gradient).  The graph plan (CSR
build) is outside the timed region, as DGL's cached CSC is.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--graph S2|S1|S1u|arxiv] [--agg sum|mean|sym]
                  [--dtype f32|bf16|f16] [--workload cfg4|cfg1|cfg2|cfg3|cfg5]

* ``--gpus N`` with N > 1 and no WORLD_SIZE in the environment: this process starts
  ``torch.distributed.run`` with N ranks (before touching the GPU) and exits with its status;
  under torchrun (WORLD_SIZE set) it is one rank.  cfg4 at N > 1 = dst-range edge-cut of the SAME
  graph (strong scaling) with a sparse RCCL all-to-all of halo K rows forward and its transpose
  for dK backward (``sirgcn.dist``); cfg5 at N > 1 = data parallel (a different 64-molecule batch
  per rank, DDP gradient all-reduce over RCCL; weak scaling).
* Without a GPU (``--dist-backend gloo``) the edge-cut plumbing is rehearsed on the CPU with the
  test-only CPU edge backend: the line is marked ``"rehearsal"`` and measures nothing.

Prints ONE JSON line (rank 0).  ``roofline``: the forward edge-aggregation kernel (the kernel the
north star names), SURVEY §8(d) algorithmic bytes ÷ its mean launch time from HIP events on the
launching stream; plus the PMC-counter and unique-bytes views and a streaming-copy rate measured in
the same process.  ``cpu_baseline``: the reference CPU dataflow restated in ``oracle/`` (DGL
edge-UDF path: gathers + index_add, torch autograd) on the S1 graph, host cores stated.
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))
sys.path.insert(0, ROOT)

METRIC = "edges/sec SIRConv fwd+bwd, d_hidden=256, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
FP32_PEAK_TFLOPS = 157.3    # fp32 MFMA = vector peak (no xf32 on gfx950)
FP16_PEAK_FLOPS = 2.5e15    # dense fp16/bf16 MFMA (MI355X_MICROARCH.md; the 5 PF figure is 2:1 sparse)
SIZEOF = {"f32": 4, "bf16": 2, "f16": 2}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfg4", choices=["cfg1", "cfg2", "cfg3", "cfg4", "cfg5"])
    ap.add_argument("--graph", default="S2", help="cfg4 graph: S2 (default), S1, S1u, arxiv")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--agg", default="sum", choices=["sum", "mean", "sym", "max"],
                    help="max: the fused per-edge W_R + running max (sirgcn.edgemlp), an MFMA-bound kernel")
    ap.add_argument("--max-bwd", default="hybrid", choices=["hybrid", "materialised", "routed"],
                    help="agg max: the default hybrid backward (routed dQ / dK passes, dW_R with the activations "
                         "recomputed: no [E, *] buffer), the edge-materialised one (EdgeMaxLinear.hybrid_bwd = "
                         "False) or the fully routed one (sirgcn.edgemlp.EdgeMaxLinear.sparse_bwd)")
    ap.add_argument("--dtype", default=None, choices=["f32", "bf16", "f16"],
                    help="feature dtype (16-bit = the autocast path); default f32 (cfg2: bf16)")
    ap.add_argument("--chunk", type=int, default=None)
    ap.add_argument("--dropout", type=float, default=None,
                    help="SIRConv feat_dropout (Q/K dropout, conv.py:60-61) in training mode; default: 0 for cfg4, "
                         "the reference's trained value for the stack workloads (cfg3 / cfg5: 0.2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-graph", default="S1", help="graph of the reference CPU dataflow baseline")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="repeat CPU baseline steps until this long")
    ap.add_argument("--no-aux", action="store_true", help="skip the copy-rate and torch-GEMM A/B measurements")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) for real runs; gloo to rehearse N ranks (CPU without a GPU)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the edge-cut (sirgcn.dist) code path even at world size 1")
    ap.add_argument("--no-capture", action="store_true",
                    help="stack workloads: launch every kernel from Python instead of replaying a captured HIP graph")
    ap.add_argument("--no-dual", action="store_true",
                    help="A/B only: the two backward edge passes as two launches instead of one")
    ap.add_argument("--torch-gemm", action="store_true",
                    help="A/B only: projections on torch fp32 GEMMs instead of the native MFMA kernels")
    ap.add_argument("--pmc-file", default=None,
                    help="PMC traffic summary (tools/pmc_traffic.py); default profiles/pmc_traffic_<graph>.json")
    return ap.parse_args()


# ------------------------------------------------------------------------------ launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def self_launch(args):
    """``bench.py --gpus N`` outside torchrun: start N ranks (one per GPU) as a child
    ``torch.distributed.run`` — before this process initialises any GPU — and return its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------------ accounting
def edge_pass_bytes(name, V_rows, E, H, agg, masked, s=4, si=4):
    """Bytes one launch of each edge pass moves in THIS design (includes the sign
    mask of the ReLU-family backward).  Recompute mode (any sigma): fwd gathers K[u]; dQ pass
    re-gathers K[u]; dK pass gathers Q[v] and G[v].  Sign-mask mode: fwd also writes H bits/edge;
    dQ pass reads only the mask; dK pass gathers G[v] + the edge's mask words (+ its permutation)."""
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


def fwd_algorithmic_bytes(V, E, H, s=4, si=4):
    """SURVEY §8(d) B_fwd = E (s_i + H s) + V (2 H s + s_i): col + K[u] per edge, Q read + S write +
    rowptr per destination (implementation-neutral: no sign mask, no sym norms)."""
    return E * (si + H * s) + V * (2 * H * s + si)


def fwd_unique_bytes(V_src, V, E, H, s=4, si=4):
    """Lower bound: every K row read ONCE (as if the gathers all hit cache after the first)."""
    return V_src * H * s + E * si + V * (2 * H * s + si)


# ------------------------------------------------------------------------------ baselines
def copy_rate(dev, nbytes=4 << 30, reps=10):
    """Streaming-copy GB/s in this process (read + write bytes / time), the achievable HBM rate."""
    import torch
    n = nbytes // 4
    a = torch.empty(n, dtype=torch.float32, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    b.copy_(a)
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        b.copy_(a)
    e1.record(st)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    del a, b
    torch.cuda.empty_cache()
    return round(2 * nbytes / (ms * 1e-3) / 1e9, 1)


def cpu_baseline(args, H):
    """The reference CPU dataflow (oracle.reference_cpu_step: DGL edge-UDF gathers + index_add,
    torch autograd) on ``--cpu-graph`` (S1 by default, one step, unchunked), rank 0 only."""
    import torch
    from torch import nn
    import oracle
    from sirgcn.synth import NAMED, powerlaw_edges
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    Vs, Es, alpha = NAMED[args.cpu_graph]
    agg = args.agg

    def setup(V, E):
        src, dst = powerlaw_edges(V, E, alpha, seed=0)
        X = torch.randn(V, H, generator=torch.Generator().manual_seed(3))
        torch.manual_seed(4)
        m = nn.ModuleList([nn.Linear(H, H), nn.Linear(H, H, bias=False), nn.Linear(H, H)])
        dY = torch.randn(V, H, generator=torch.Generator().manual_seed(5))
        w = [m[0].weight.data, m[0].bias.data, m[1].weight.data, m[2].weight.data, m[2].bias.data]
        return src, dst, X, w, dY

    src, dst, X, w, dY = setup(Vs // 50, Es // 50)            # warm-up on a 2% sample (allocator, threads)
    oracle.reference_cpu_step(src, dst, Vs // 50, X, *w, dY, agg, "leaky", 0.2)
    src, dst, X, w, dY = setup(Vs, Es)
    n, t0 = 0, time.perf_counter()
    while True:
        oracle.reference_cpu_step(src, dst, Vs, X, *w, dY, agg, "leaky", 0.2)
        n += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or n >= 5:
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
    return {"value": round(Es * n / el, 1), "unit": "edges/s", "cores": cores, "kind": "port",
            "sample": f"{args.cpu_graph}: Chung-Lu alpha={alpha} V={Vs} E={Es} H={H} {agg} LeakyReLU(0.2), "
                      f"{n} full fwd+bwd step(s) in {el:.1f}s, unchunked (oracle.reference_cpu_step: DGL edge-UDF "
                      f"dataflow, torch CPU autograd)",
            "cpu_model": cpu_model}


# ------------------------------------------------------------------------------ timing
def kernel_table(timing, rows_of, edges, H, agg, masked, s):
    import torch  # noqa: F401
    kernels, gemm = {}, {}
    for name, evs in timing.items():
        t = sum(a.elapsed_time(b) for a, b, _ in evs) / len(evs)    # ms per launch
        if name.startswith("sir_gemm_"):       # MFMA-bound projections: flops (and HBM bytes) per launch
            if name.startswith("sir_gemm_pack"):
                continue
            fl = sum(w[0] for _, _, w in evs) / len(evs)
            by = sum(w[1] for _, _, w in evs) / len(evs)
            gemm[name] = {"ms": round(t, 4), "launches": len(evs), "flops": fl,
                          "TFLOPs": round(fl / (t * 1e-3) / 1e12, 1), "hbm_bytes": by,
                          "GBps": round(by / (t * 1e-3) / 1e9, 1),
                          # fp16/bf16 MFMAs issued per product: 3 for the two-term split, 1 for 16-bit operands
                          "mfma_per_product": 1 if name.split(" ")[0].endswith("16") else 3}
            continue
        if name == "sir_edge_mlp_fwd":         # fused per-edge dense layer: fp32-equivalent flops per launch
            fl = sum(w for _, _, w in evs) / len(evs)
            kernels[name] = {"ms": round(t, 4), "launches": len(evs), "flops": fl,
                             "TFLOPs": round(fl / (t * 1e-3) / 1e12, 2)}
            continue
        if not name.startswith("sir_edge_agg"):
            kernels[name] = {"ms": round(t, 4), "launches": len(evs)}
            continue
        if name == "sir_edge_agg_bwd":         # both backward passes in one launch (MEAN: on G / deg)
            b = sum(edge_pass_bytes(n, rows_of(n), edges, H, "sum" if agg == "mean" else agg, masked, s=s)
                    for n in ("sir_edge_agg_bwd_dst", "sir_edge_agg_bwd_src"))
        else:
            b = edge_pass_bytes(name, rows_of(name), edges, H, agg, masked, s=s)
        kernels[name] = {"ms": round(t, 4), "launches": len(evs), "design_bytes": b,
                         "GBps": round(b / (t * 1e-3) / 1e9, 1)}
    return kernels, gemm


STEP_MS = []       # per-step times (ms) of the last timed_loop, from HIP events between steps


def timed_loop(step, steps, warmup, world, dist, dev):
    """Time EXACTLY ``steps`` steps between barrier + synchronize; per-step HIP events on the
    current stream (no host sync inside the loop) give the median beside the mean."""
    import torch
    from sirgcn import _native
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    timing = _native.enable_timing(True)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(steps):
        step()
        evs[i + 1].record()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    _native.enable_timing(False)
    STEP_MS[:] = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]
    return el, timing


def median(xs):
    xs = sorted(xs)
    n = len(xs)
    return (xs[n // 2] if n % 2 else 0.5 * (xs[n // 2 - 1] + xs[n // 2])) if n else None


def max_over_ranks(x, world, dist, dev):
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


# ------------------------------------------------------------------------------ main
def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))

    import torch
    import torch.distributed as dist
    from torch import nn

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rehearsal = not torch.cuda.is_available()
    if rehearsal:
        if args.dist_backend != "gloo" or args.workload not in ("cfg4", "cfg5"):
            raise SystemExit("no GPU: only the cfg4 edge-cut and cfg5 data-parallel plumbing can be rehearsed "
                             "(--dist-backend gloo)")
        dev = torch.device("cpu")
        torch.set_num_threads(max(1, min(4, os.cpu_count() // max(world, 1))))
    else:
        ndev = torch.cuda.device_count()
        dev = torch.device("cuda", local % max(ndev, 1))     # one rank per GPU (wraps only in rehearsals)
        torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    if args.workload == "cfg4":
        out = run_edge_cut(args, world, rank, dev, rehearsal, torch, dist, nn)
    elif rehearsal:
        out = rehearse_stack(args, world, rank, dev, torch, dist)
    else:
        out = run_stack(args, world, rank, dev, torch, dist)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_edge_cut(args, world, rank, dev, rehearsal, torch, dist, nn):
    from sirgcn import SIRConv, _native, linalg
    from sirgcn.conv import EdgeAggregate
    if args.torch_gemm:
        linalg.USE_NATIVE = False
    if args.no_dual:
        EdgeAggregate.dual = False
    from sirgcn.graph import DEFAULT_CHUNK
    from sirgcn.synth import NAMED, powerlaw_edges
    H = args.hidden
    dtn = args.dtype or "f32"
    dt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[dtn]
    V, E, alpha = NAMED[args.graph]
    src, dst = powerlaw_edges(V, E, alpha, seed=0)

    torch.manual_seed(4)
    p_drop = args.dropout or 0.0
    conv = SIRConv(H, H, H, nn.LeakyReLU(0.2, inplace=True), p_drop, agg_type=args.agg).to(dev)
    if args.agg == "max" and args.max_bwd != "hybrid":
        from sirgcn.edgemlp import EdgeMaxLinear
        if args.max_bwd == "routed":
            EdgeMaxLinear.sparse_bwd = True
        else:
            EdgeMaxLinear.hybrid_bwd = False
    if args.chunk:
        conv.chunk = args.chunk
    X_full = torch.randn(V, H, generator=torch.Generator().manual_seed(3))
    dY_full = torch.randn(V, H, generator=torch.Generator().manual_seed(5))

    dconv = None
    if world == 1 and not args.force_dist and not rehearsal:
        from sirgcn import Graph
        g = Graph(src, dst, V)
        X = X_full.to(dev).requires_grad_(True)
        dY = dY_full.to(dev)
        layer = lambda: conv(g, X)
        rows_local, edges_local, rows_src = V, E, V
    else:
        from sirgcn.dist import DistGraph, DistSIRConv
        backend = None
        if rehearsal:          # test-only CPU edge passes (tests/cpu_edge_backend.py): plumbing, not a measurement
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import cpu_edge_backend as backend
        dg = DistGraph.from_global(src, dst, V, rank, world, dev, chunk=args.chunk or DEFAULT_CHUNK)
        # weight gradients all-reduced inside the backward, dW_R / dW_Q under the reverse exchange
        dconv = DistSIRConv(conv, backend=backend, reduce_in_backward=True)
        r0, r1 = dg.row_begin, dg.row_end
        X = X_full[r0:r1].to(dev).requires_grad_(True)
        dY = dY_full[r0:r1].to(dev)
        layer = lambda: dconv(dg, X)
        rows_local, edges_local, rows_src = r1 - r0, dg.num_local_edges, dg.n_ext
    del X_full, dY_full

    # the incoming gradient in the dtype of Y (a 16-bit tensor under autocast: the gradient a
    # downstream autocast layer hands back), cast once outside the timed region
    dY_in = dY if dt == torch.float32 else dY.to(dt)

    def step():
        conv.zero_grad(set_to_none=True)
        X.grad = None
        if dt != torch.float32:
            with torch.autocast(dev.type, dtype=dt):
                Y = layer()
        else:
            Y = layer()
        Y.backward(dY_in if dY_in.dtype == Y.dtype else dY_in.to(Y.dtype))
        if dconv is not None:
            dconv.allreduce_grads()

    if rehearsal:
        el, timing = rehearsal_loop(step, args.steps, args.warmup, world, dist)
    else:
        el, timing = timed_loop(step, args.steps, args.warmup, world, dist, dev)
    el = max_over_ranks(el, world, dist, dev if args.dist_backend == "nccl" and not rehearsal else "cpu")
    med = None if rehearsal else max_over_ranks(median(STEP_MS), world, dist,
                                                dev if args.dist_backend == "nccl" else "cpu")
    ms = 1e3 * el / args.steps
    out = {"metric": METRIC, "value": round(E / (el / args.steps), 1), "unit": "edges/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": dtn, "data": "synthetic",
           "config": {"workload": f"cfg4 {args.graph}: Chung-Lu power-law V={V} E={E} alpha={alpha}; 1 SIRConv layer "
                                  f"d_in=H=d_out={H}, agg={args.agg}, LeakyReLU(0.2), {dtn}, feat_dropout={p_drop}"
                                  f"{' (autocast)' if dtn != 'f32' else ''}; fwd+bwd incl. projections",
                      "graph": args.graph, "V": V, "E": E, "hidden": H, "agg": args.agg, **({"max_bwd": args.max_bwd} if args.agg == "max" else {}),
                      "parallelism": f"edge-cut dst-range x{world}, pipelined sparse halo all-to-alls" if world > 1
                      else "single GPU"}}
    if rehearsal:
        out["rehearsal"] = ("CPU gloo rehearsal of the launcher / partition / exchange plumbing; edge passes on "
                            "the test-only CPU backend: NOT a measurement")
        out["n_gpus"] = world
        return out

    # the median of the per-step HIP-event times; value / ms_per_step stay the mean over
    # the bracketed K steps (the bench contract)
    out["ms_per_step_median"] = round(med, 3)
    out["value_median"] = round(E / (med * 1e-3), 1)
    from sirgcn.conv import EdgeAggregate
    s = SIZEOF[dtn]
    masked = bool(EdgeAggregate.use_mask and _native.mask_words(H, _native.ACT_LEAKY)) and args.agg != "max"
    kernels, gemm = kernel_table(timing, lambda n: rows_src if n == "sir_edge_agg_bwd_src" else rows_local,
                                 edges_local, H, args.agg, masked, s)
    if "sir_edge_mlp_fwd" in kernels:      # max: the per-edge W_R GEMM bounds the dominant kernel
        k = kernels["sir_edge_mlp_fwd"]
        # fp32: split-fp16 MFMA (3 fp16 MFMAs per fp32-accurate product): the peak in fp32-equivalent
        # flops is the dense fp16 peak / 3.  Under autocast the 16-bit forward (sir_edge_mlp_fwd*_st)
        # runs ONE 16-bit MFMA per product: its peak is the dense 16-bit peak itself.
        from sirgcn import edgemlp
        per = 1 if (dtn in ("bf16", "f16") and edgemlp.NATIVE_16) else 3
        peak = FP16_PEAK_FLOPS / per / 1e12
        form = "one 16-bit MFMA per product" if per == 1 else "split-fp16 MFMA, 3 per product"
        out["roofline"] = {"bound": "mfma", "kernel": f"sir_edge_mlp_fwd (gather -> sigma -> {form} W_R -> running max)",
                           "achieved": k["TFLOPs"], "peak": round(peak, 1), "unit": "TFLOP/s",
                           "frac": round(k["TFLOPs"] / peak, 4), "traffic": None,
                           "flops_formula": f"2 * E * H * O per launch ({'16-bit' if per == 1 else 'fp32-equivalent'}; "
                                            f"{per} v_mfma_f32_32x32x16 per product)",
                           "fp16_mfma_util": round(per * k["TFLOPs"] * 1e12 / FP16_PEAK_FLOPS, 4),
                           "vs_fp32_mfma_peak": round(k["TFLOPs"] / FP32_PEAK_TFLOPS, 4),
                           "ms_per_launch": k["ms"]}
    else:
        out["roofline"] = roofline_fwd(args, kernels, rows_local, edges_local, rows_src, H, s, world)
    out["roofline"]["all_kernels"] = kernels
    if gemm:
        out["projections"] = projections(gemm, args.steps)
    out["design_bytes_per_step"] = design_bytes(kernels, gemm, args.steps, ms)
    if dconv is not None:     # halo exchange volume per rank (rows of H), max over ranks
        ex = torch.tensor([dg.n_halo, dg.exchange_rows()[1], edges_local], dtype=torch.float64,
                          device=dev if args.dist_backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(ex, op=dist.ReduceOp.MAX)
        out["exchange"] = {"halo_rows_max": int(ex[0]), "send_rows_max": int(ex[1]), "local_edges_max": int(ex[2]),
                           "bytes_per_direction_max": int(ex[0]) * H * s, "exchange_chunks": dg.chunks,
                           "dense_allgather_rows": V - min(dg.bounds[i + 1] - dg.bounds[i] for i in range(world))}
    if world == 1 and not args.no_aux:
        out["roofline"]["copy_GBps_measured"] = copy_rate(dev)
        if not args.torch_gemm and dtn == "f32":        # IEEE fp32 projections (torch / hipBLASLt) beside it
            linalg.USE_NATIVE = False
            el2, _ = timed_loop(step, max(3, args.steps // 4), 2, 1, dist, dev)
            linalg.USE_NATIVE = True
            out["ms_per_step_torch_fp32_gemm"] = round(1e3 * el2 / max(3, args.steps // 4), 3)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, H)
    return out


def rehearsal_loop(step, steps, warmup, world, dist):
    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    return el, {}


def roofline_fwd(args, kernels, V, E, V_src, H, s, world):
    """The forward edge-aggregation kernel against HBM: §8(d) algorithmic bytes / HIP-event time."""
    k = kernels["sir_edge_agg_fwd"]
    t = k["ms"] * 1e-3
    alg = fwd_algorithmic_bytes(V, E, H, s)
    uniq = fwd_unique_bytes(V_src, V, E, H, s)
    ach = alg / t / 1e9
    traffic = None
    traffic_source = None
    dts = args.dtype or "f32"
    pmc_file = args.pmc_file or os.path.join(ROOT, "profiles", f"pmc_traffic_{args.graph}"
                                             f"{'' if dts == 'f32' else '_' + dts}.json")
    try:
        with open(pmc_file) as f:
            pmc = json.load(f)
        rec = pmc.get("kernels", {}).get("sir_edge_agg_fwd")
        if (rec and world == 1 and pmc.get("graph") == args.graph and pmc.get("agg") == args.agg
                and pmc.get("H") == H and pmc.get("dtype", "f32") == (args.dtype or "f32")):
            traffic = rec["hbm_bytes_per_launch"]      # L2<->fabric bytes (Infinity-Cache hits included)
            # which build the counters were taken on, against the build being timed: the counter
            # bytes stand while the edge kernels' sources are unchanged
            from sirgcn import _native
            took = pmc.get("build") or {}
            now = _native.build_id()
            traffic_source = {"file": os.path.relpath(pmc_file, ROOT), "counters_build": took or "not recorded",
                              "timed_build": now,
                              "same_edge_kernels": (took.get("edge_source_hash") == now["edge_source_hash"])
                              if took else None}
    except (OSError, ValueError):
        pass
    frac_alg = ach / HBM_PEAK_GBS
    # The physical figure is the HBM-side one: counter bytes (PMC FETCH_SIZE x2 + WRITE_SIZE, a
    # separate profiled run of this build: profiles/pmc_traffic_<graph>.json) / this launch time.
    # Without it, the algorithmic figure is reported as is — never capped: on power-law graphs the
    # hub rows are served by L2 / Infinity Cache, so the algorithmic rate can exceed the HBM peak.
    phys = traffic / t / 1e9 if traffic else None
    out = {"bound": "hbm", "kernel": "sir_edge_agg_fwd (k_edge<FWD> + k_combine)",
           "achieved": round(phys if phys else ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round((phys if phys else ach) / HBM_PEAK_GBS, 4),
           "frac_basis": ("counter: L2-miss bytes from PMC (FETCH_SIZE x2 + WRITE_SIZE); FETCH_SIZE also counts "
                          "Infinity-Cache (MALL) hits, so this is an upper bound on physical HBM bytes")
                         if phys else "algorithmic (no PMC file for this config)",
           "traffic": traffic, "traffic_source": traffic_source, "algorithmic_bytes": alg, "ms_per_launch": k["ms"],
           "achieved_algorithmic": round(ach, 1), "frac_algorithmic": round(frac_alg, 4),
           "bytes_formula": "SURVEY 8(d): E*(s_i + H*s) + V*(2*H*s + s_i)",
           "unique_bytes": uniq, "frac_unique": round(uniq / t / 1e9 / HBM_PEAK_GBS, 4),
           "frac_counter": round(phys / HBM_PEAK_GBS, 4) if phys else None}
    if frac_alg > 1.0:
        out["note"] = "algorithmic rate above the HBM peak: cache-served gathers (see frac_unique / frac_counter)"
    return out


def projections(gemm, steps):
    """``fp16_mfma_util``: the 16-bit MFMA work actually issued (flops x MFMAs per product: 3 for the
    split-fp16 fp32 kernels, 1 for the bf16 / fp16 kernels) / time / the dense fp16 peak."""
    fl = sum(g["flops"] * g["launches"] for g in gemm.values()) / steps
    fl16 = sum(g["flops"] * g["launches"] * g["mfma_per_product"] for g in gemm.values()) / steps
    by = sum(g["hbm_bytes"] * g["launches"] for g in gemm.values()) / steps
    tg = sum(g["ms"] * g["launches"] for g in gemm.values()) / steps
    return {"bound": "mfma", "ms_per_step": round(tg, 3), "flops_per_step": fl,
            "achieved_fp32_equiv_TFLOPs": round(fl / (tg * 1e-3) / 1e12, 1),
            "fp16_mfma_util": round(fl16 / (tg * 1e-3) / FP16_PEAK_FLOPS, 4),
            "vs_fp32_peak": round(fl / (tg * 1e-3) / (FP32_PEAK_TFLOPS * 1e12), 3),
            "hbm_bytes_per_step": by, "hbm_frac": round(by / (tg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "kernels": gemm}


def design_bytes(kernels, gemm, steps, ms):
    """Bytes one step moves in THIS design: edge passes (incl. the sign mask) + the
    projection GEMMs' A, B and C; ÷ the step time = the whole step's HBM rate."""
    e = sum(k.get("design_bytes", 0) * k["launches"] for k in kernels.values()) / steps
    g = sum(k["hbm_bytes"] * k["launches"] for k in gemm.values()) / steps
    return {"edge_passes": e, "projections": g, "total": e + g,
            "GBps_over_step": round((e + g) / (ms * 1e-3) / 1e9, 1)}


def rehearse_stack(args, world, rank, dev, torch, dist):
    """cfg5 without a GPU: the same per-rank batches, DDP wrapper and gloo all-reduce as the RCCL run,
    with the test-only CPU stand-ins of the conv / norm modules (tests/cpu_stack_modules.py): a
    rehearsal of the launcher and the data-parallel plumbing, not a measurement."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import cpu_stack_modules as cpu
    from sirgcn.workloads import CONFIGS, dp_replica
    name = args.workload
    c = CONFIGS[name]
    p_drop = c["feat_dropout"] if args.dropout is None else args.dropout
    model, stack, g, X, dY = dp_replica(name, rank, world, dev, cpu.SIRConv, cpu.GraphNorm, feat_dropout=p_drop)
    X.requires_grad_(True)

    def step():
        model.zero_grad(set_to_none=True)
        X.grad = None
        model(g, X).backward(dY)

    el, _ = rehearsal_loop(step, args.steps, args.warmup, world, dist)
    tot = torch.tensor([g.num_edges(), g.num_nodes(), g.batch_size], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tot)
    E_all, V_all, B_all = (int(x) for x in tot.tolist())
    return {"metric": "layer-edges/sec SIRConv stack fwd+bwd (E x layers / step time)",
            "value": round(E_all * c["layers"] / (el / args.steps), 1), "unit": "edges/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{name}: {dict(c, feat_dropout=p_drop)} per rank, DDP over gloo",
                       "V_total": V_all, "E_total": E_all, "graphs": B_all,
                       "parallelism": f"data-parallel x{world}"},
            "rehearsal": "CPU gloo rehearsal of the launcher / per-rank batches / DDP all-reduce plumbing with the "
                         "test-only CPU stand-in modules (tests/cpu_stack_modules.py); measures nothing"}


def run_stack(args, world, rank, dev, torch, dist):
    """BASELINE configs 1/2/3/5: the reference models' layer loops (sirgcn.workloads)."""
    from sirgcn import GraphNorm, SIRConv, _native
    from sirgcn.workloads import CONFIGS, DTYPES, dp_replica
    name = args.workload
    c = CONFIGS[name]
    dtn = args.dtype or c["dtype"]
    dt = DTYPES[dtn]
    if world > 1 and name != "cfg5":
        raise SystemExit(f"{name} is a single-GPU workload (cfg5 is the data-parallel one, cfg4 the edge-cut)")
    p_drop = c["feat_dropout"] if args.dropout is None else args.dropout
    # DP replicas: a different batch per rank, RCCL gradient all-reduce (DDP)
    model, stack, g, X, dY = dp_replica(name, rank, world, dev, SIRConv, GraphNorm, feat_dropout=p_drop)
    X.requires_grad_(True)
    dY_in = dY if dt == torch.float32 else dY.to(dt)      # cast outside the timed region (as in run_edge_cut)

    def step():
        model.zero_grad(set_to_none=True)
        X.grad = None
        if dt != torch.float32:
            with torch.autocast("cuda", dtype=dt, cache_enabled=False):
                Y = model(g, X)
        else:
            Y = model(g, X)
        Y.backward(dY_in if dY_in.dtype == Y.dtype else dY_in.to(Y.dtype))

    # Batched small graphs are launch-bound (SURVEY §7 "tiny batched graphs"): at N = 1 the whole
    # fwd+bwd step (every kernel, every ctypes launch, the allocator's work) is captured once into
    # a HIP graph and replayed; per-kernel HIP-event timing is then measured on the eager step.
    captured = None
    if world == 1 and not args.no_capture:
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(3):
                step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        captured = torch.cuda.CUDAGraph()
        with torch.cuda.graph(captured):
            step()
        torch.cuda.synchronize(dev)
    if captured is not None:
        _, timing = timed_loop(step, 3, 1, world, dist, dev)          # eager: per-kernel events
        el, _ = timed_loop(captured.replay, args.steps, args.warmup, world, dist, dev)
    else:
        el, timing = timed_loop(step, args.steps, args.warmup, world, dist, dev)
    el = max_over_ranks(el, world, dist, dev)
    med = max_over_ranks(median(STEP_MS), world, dist, dev)
    L, H, E, V = c["layers"], c["hidden"], g.num_edges(), g.num_nodes()
    tot = torch.tensor([E, V, g.batch_size], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tot)
    E_all, V_all, B_all = (int(x) for x in tot.tolist())
    from sirgcn.conv import EdgeAggregate
    masked = bool(EdgeAggregate.use_mask and _native.mask_words(H, _native.ACT_LEAKY))
    kernels, gemm = kernel_table(timing, lambda n: V, E, H, c["agg"], masked, SIZEOF[dtn])
    eager_steps = 3 if captured is not None else args.steps
    out = {"metric": "layer-edges/sec SIRConv stack fwd+bwd (E x layers / step time)",
           "value": round(E_all * L / (el / args.steps), 1), "unit": "edges/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 3),
           "higher_is_better": True, "scaling": "weak" if name == "cfg5" else "strong", "vs_baseline": None,
           "dtype": dtn, "data": "synthetic",
           "config": {"workload": f"{name}: {dict(CONFIGS[name], feat_dropout=p_drop)} V={V} E={E} graphs={g.batch_size}"
                                  f"{' per rank, DDP over RCCL' if world > 1 else ''}",
                      "graphs_per_s": round(B_all / (el / args.steps), 1), "V_total": V_all, "E_total": E_all,
                      "parallelism": f"data-parallel x{world}" if world > 1 else "single GPU"},
           "ms_per_step_median": round(med, 3), "kernels": kernels, "hip_graph": captured is not None}
    if captured is not None:
        out["kernels_note"] = "per-kernel times from 3 eager steps; value / ms_per_step from the replayed HIP graph"
    if gemm:
        out["projections"] = projections(gemm, eager_steps)
    return out


if __name__ == "__main__":
    main()

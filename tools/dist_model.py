#!/usr/bin/env python3
"""Per-rank step model of the edge-cut layer (sirgcn/dist.py) at W ranks on the S2 graph.

    python tools/dist_model.py [--world 8] [--chunks 4] [--link-GBps 153] [--graph S2]

Two resources per rank — the compute stream (kernels in the order DistSIRConvFunction issues them)
and the xGMI wire (RCCL's alltoallv chunks, in order, each taking the bottleneck link's bytes /
link bandwidth) — and the dependencies of dist.py between them:

forward : K GEMM -> pack chunk c (index_select of the rows peers need) -> wire chunk c;  Q GEMM,
          own-source segment; segment c+1 after wire chunk c (edge pass + read-modify-write of S);
          Y GEMM.
backward: G GEMM -> dK over halo chunk c -> reverse wire chunk c;  one-launch dQ || own-row dK;
          dW_R, dX_Q = dQ W_Q, dW_Q under the wire;  after the last chunk: dK completion (segment
          sum over own + received rows), dX += dK W_K, dW_K, the weight-gradient all-reduce.

Kernel times are the single-GPU S2 kernels scaled by each rank's share of the work (edges for the
edge passes, rows for the GEMMs): the measured r03 final profile (profiles/r03_final_S2_kernel_summary.txt)
unless overridden.  Pass-through kernels (pack, RMW, completion) run at the measured streaming rate
(6.2 TB/s read+write, profiles/r03_stream_floor.txt).  Halo sizes, per-peer rows and per-chunk edge
counts come from the real partition of the synthetic graph (sirgcn.synth, partition_rows).

The link bandwidth is the task statement's figure (7 xGMI links x ~153 GB/s per GPU), read as per
direction; --link-GBps 76.5 gives the model with half of it per direction."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))

# single-GPU S2 kernel times (ms), r03 final profile: k_edge fwd + k_combine, k_edge_mask_dual, the
# persistent NT GEMMs (QK N=512 K=256; Y, G N=256; dX K=512) and the TN GEMMs (dW_R; [dW_Q; dW_K])
SINGLE = {"fwd": 5.77, "bwd": 6.82, "QK": 2.03, "Y": 0.98, "G": 0.98, "dX": 1.61, "dWR": 0.87, "dWQK": 1.91,
          "step": 20.99}
# share of the one-launch backward that is the dK (source) pass, by design bytes (dst 5.4 GB,
# src 44.6 GB of the sign-mask passes)
DK_SHARE = 44.6 / (44.6 + 5.4)


def partition_stats(graph, world, chunks, seed=0, row_weight=None):
    from sirgcn.dist import ROW_WEIGHT, partition_rows
    from sirgcn.synth import NAMED, powerlaw_edges
    V, E, a = NAMED[graph]
    src, dst = powerlaw_edges(V, E, a, seed)
    bounds = partition_rows(torch.bincount(dst, minlength=V), world, ROW_WEIGHT if row_weight is None else row_weight)
    b = torch.tensor(bounds)
    owner_of = lambda x: torch.searchsorted(b, x, right=True) - 1   # noqa: E731
    order = torch.argsort(dst, stable=True)
    src_s = src[order]
    cnt = torch.bincount(owner_of(dst[order]), minlength=world)
    off = [0] + torch.cumsum(cnt, 0).tolist()
    ranks = []
    rows_pq = torch.zeros(world, world, dtype=torch.int64)
    for p in range(world):
        s = src_s[off[p]:off[p + 1]]
        own = owner_of(s)
        remote = own != p
        u, inv = torch.unique(s[remote], return_inverse=True)       # halo rows, ascending id
        uo = owner_of(u)
        per = torch.bincount(uo, minlength=world)
        rows_pq[p] = per
        # chunk of each halo row: the part of its owner's row range it lies in (sirgcn/dist.py, r05)
        lo = b[uo]
        hchunk = ((u - lo) * chunks) // (b[uo + 1] - lo)
        edges_c = torch.bincount(hchunk[inv], minlength=chunks)
        rows_c = torch.bincount(hchunk, minlength=chunks)
        # destination rows with >= 1 edge from halo chunk c: the rows segment c reads-modifies-writes
        d_own = dst[order][off[p]:off[p + 1]][remote]
        seg_rows = [int(torch.unique(d_own[hchunk[inv] == c]).numel()) for c in range(chunks)]
        ranks.append({"rows": bounds[p + 1] - bounds[p], "edges": int(s.numel()), "own_edges": int((~remote).sum()),
                      "halo": int(u.numel()), "edges_c": edges_c.tolist(), "rows_c": rows_c.tolist(),
                      "seg_rows": seg_rows})
    for p in range(world):
        ranks[p]["send"] = int(rows_pq[:, p].sum())
    return {"V": V, "E": E, "bounds": bounds, "ranks": ranks, "rows_pq": rows_pq.tolist()}


def simulate(st, world, chunks, H=256, link=153e9, stream=6.2e12, single=SINGLE, allreduce_ms=0.05,
             merge_first=False, schedule="r05"):
    """``schedule``: "r04" — K GEMM over all own rows before the first pack; dK completed, dX += dK W_K
    and dW_K after the LAST reverse chunk; every weight gradient all-reduced at the end.  "r05" (dist.py
    now) — chunks cut by the owner's row range: the K GEMM runs part by part and chunk c is packed and
    sent right after part c; part c's dK is completed as soon as reverse chunk c lands, and its dX rows
    (one K = 2H GEMM on [dQ | dK]) and dW_K share computed; dW_R / dW_Q all-reduced under the exchange,
    only dW_K's at the end."""
    if schedule == "r04":
        return _simulate_r04(st, world, chunks, H, link, stream, single, allreduce_ms, merge_first)
    V, E = st["V"], st["E"]
    rb = H * 4
    rows_pq = torch.tensor(st["rows_pq"], dtype=torch.float64)
    wire_c = float(rows_pq.max()) / chunks * rb / link * 1e3
    out = []
    for p, r in enumerate(st["ranks"]):
        fr, n = r["edges"] / E, r["rows"] / V
        t_stream = lambda by: by / stream * 1e3                   # noqa: E731
        # ---------------- forward: K part c -> pack c -> wire c
        comp, wire_free, land = 0.0, 0.0, []
        for c in range(chunks):
            comp += single["QK"] / 2 * n / chunks + t_stream(2 * r["send"] / chunks * rb)
            start = max(comp, wire_free)
            wire_free = start + wire_c
            land.append(wire_free)
        comp += single["QK"] / 2 * n                             # Q GEMM
        if merge_first:
            comp = max(comp, land[0]) + single["fwd"] * (r["own_edges"] + r["edges_c"][0]) / E
        else:
            comp += single["fwd"] * r["own_edges"] / E
        for c in range(1 if merge_first else 0, chunks):      # segment c re-reads / re-writes only its rows
            comp = max(comp, land[c]) + single["fwd"] * r["edges_c"][c] / E + t_stream(2 * r["seg_rows"][c] * rb)
        comp += single["Y"] * n
        t_fwd = comp
        # ---------------- backward
        comp = single["G"] * n
        wire_free = 0.0
        land = []
        for c in range(chunks):
            comp += single["bwd"] * DK_SHARE * r["edges_c"][c] / E
            start = max(comp, wire_free)
            wire_free = start + wire_c
            land.append(wire_free)
        comp += single["bwd"] * (1 - DK_SHARE) * fr + single["bwd"] * DK_SHARE * r["own_edges"] / E
        comp += (single["dWR"] + single["dWQK"] / 2) * n         # dW_R, dW_Q
        wire_free += allreduce_ms                                # dW_R / dW_Q all-reduce behind the chunks
        recv = sum(st["rows_pq"][q][p] for q in range(world))
        for c in range(chunks):                                  # part c as its chunk lands
            comp = max(comp, land[c])
            comp += t_stream((recv / chunks + 2 * r["rows"] / chunks) * rb)          # completion of part c
            comp += single["dX"] * n / chunks                    # dX[part] = [dQ | dK][part] [W_Q; W_K]
            comp += single["dWQK"] / 2 * n / chunks                                 # dW_K += dK^T X
        comp = max(comp, wire_free) + allreduce_ms * 0.5         # dW_K's all-reduce (a third of the bytes)
        out.append({"rank": p, "fwd_ms": round(t_fwd, 3), "bwd_ms": round(comp, 3), "step_ms": round(t_fwd + comp, 3)})
    step = max(o["step_ms"] for o in out)
    return {"world": world, "chunks": chunks, "link_GBps": link / 1e9, "wire_ms_per_chunk": round(wire_c, 3),
            "wire_ms_per_direction": round(wire_c * chunks, 3), "ranks": out, "step_ms": step,
            "single_gpu_step_ms": single["step"], "speedup": round(single["step"] / step, 2)}


def _simulate_r04(st, world, chunks, H=256, link=153e9, stream=6.2e12, single=SINGLE, allreduce_ms=0.05,
                  merge_first=False):
    """Per-rank forward / backward end times (ms) of the two-resource model; the step is the slowest rank."""
    V, E = st["V"], st["E"]
    rb = H * 4                                                   # bytes of one fp32 row
    rows_pq = torch.tensor(st["rows_pq"], dtype=torch.float64)
    # wire time of chunk c: the busiest link (peer pair) moves its 1/chunks share of the rows
    wire_c = float(rows_pq.max()) / chunks * rb / link * 1e3
    out = []
    for p, r in enumerate(st["ranks"]):
        fr, n = r["edges"] / E, r["rows"] / V
        t_stream = lambda by: by / stream * 1e3                   # noqa: E731
        # ---------------- forward
        comp = single["QK"] / 2 * n                              # K GEMM (own rows)
        wire_free = 0.0
        land = []
        for c in range(chunks):
            comp += t_stream(2 * r["send"] / chunks * rb)         # pack chunk c (read + write)
            start = max(comp, wire_free)
            wire_free = start + wire_c
            land.append(wire_free)
        comp += single["QK"] / 2 * n                             # Q GEMM
        if merge_first:      # own-source edges and chunk 0's in ONE segment (one read-modify-write fewer)
            comp = max(comp, land[0]) + single["fwd"] * (r["own_edges"] + r["edges_c"][0]) / E
        else:
            comp += single["fwd"] * r["own_edges"] / E           # own-source segment (writes S)
        for c in range(1 if merge_first else 0, chunks):
            comp = max(comp, land[c]) + single["fwd"] * r["edges_c"][c] / E + t_stream(2 * r["rows"] * rb)
        comp += single["Y"] * n
        t_fwd = comp
        # ---------------- backward
        comp = single["G"] * n
        wire_free = 0.0
        for c in range(chunks):
            comp += single["bwd"] * DK_SHARE * r["edges_c"][c] / E
            start = max(comp, wire_free)
            wire_free = start + wire_c
        comp += single["bwd"] * (1 - DK_SHARE) * fr + single["bwd"] * DK_SHARE * r["own_edges"] / E
        comp += (single["dWR"] + single["dX"] / 2 + single["dWQK"] / 2) * n
        comp = max(comp, wire_free)
        comp += t_stream((r["halo"] * 0 + sum(st["rows_pq"][q][p] for q in range(world)) + 2 * r["rows"]) * rb)
        comp += single["dX"] / 2 * n + t_stream(2 * r["rows"] * rb)   # dX += dK W_K (read-modify-write)
        comp += single["dWQK"] / 2 * n + allreduce_ms
        out.append({"rank": p, "fwd_ms": round(t_fwd, 3), "bwd_ms": round(comp, 3), "step_ms": round(t_fwd + comp, 3)})
    step = max(o["step_ms"] for o in out)
    # compute-only floor (wire infinitely fast) of the slowest rank, for the attribution
    return {"world": world, "chunks": chunks, "link_GBps": link / 1e9, "wire_ms_per_chunk": round(wire_c, 3),
            "wire_ms_per_direction": round(wire_c * chunks, 3), "ranks": out, "step_ms": step,
            "single_gpu_step_ms": single["step"], "speedup": round(single["step"] / step, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="S2")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--chunks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--link-GBps", type=float, nargs="+", default=[153.0, 76.5])
    ap.add_argument("--single-json", help="per-kernel single-GPU ms (keys of SINGLE) to replace the r03 profile")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    single = dict(SINGLE)
    if a.single_json:
        with open(a.single_json) as f:
            single.update(json.load(f))
    res = {"graph": a.graph, "single_gpu_kernels_ms": single, "models": []}
    for C in a.chunks:
        st = partition_stats(a.graph, a.world, C)
        if "partition" not in res:
            res["partition"] = {"halo_rows": [r["halo"] for r in st["ranks"]],
                                "send_rows": [r["send"] for r in st["ranks"]],
                                "own_edges": [r["own_edges"] for r in st["ranks"]],
                                "rows": [r["rows"] for r in st["ranks"]],
                                "busiest_link_rows": max(max(x) for x in st["rows_pq"])}
        for L in a.link_GBps:
            for sched in ("r04", "r05"):
                m = simulate(st, a.world, C, link=L * 1e9, single=single, merge_first=True, schedule=sched)
                res["models"].append({k: m[k] for k in ("chunks", "link_GBps", "wire_ms_per_direction", "step_ms",
                                                        "speedup")}
                                     | {"schedule": sched, "merge_first": True,
                                        "slowest": max(m["ranks"], key=lambda o: o["step_ms"])})
                print(json.dumps(res["models"][-1]))
    print(json.dumps(res["partition"]))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Turn two rocprofv3 counter passes into per-launch HBM bytes of each SIRConv edge pass.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --graph S2 --agg sum --H 256

Corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and WRITE_SIZE are
KiB (x1024); on gfx950 FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced
read, so reads are doubled (every gather in these kernels is a 16 B/lane load; the 8 B sign-mask
words are the uncalibrated remainder).  WRITE_SIZE is exact for 16 B/lane stores.  A
``k_combine`` dispatch (split-row tail) is attributed to the edge pass dispatched just before it,
so a "launch" is the whole ABI call, as bench.py times it.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

def build_id():
    """The library / edge-kernel source hashes of the tree the counters were taken on (bench.py
    names them beside the traffic it reads from this file)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sir-gcn_amd"))
    from sirgcn import _native
    return _native.build_id()


PASSES = {0:"sir_edge_agg_fwd", 1: "sir_edge_agg_bwd_dst", 2: "sir_edge_agg_bwd_src"}


def pass_of(short):
    """ABI call of an edge kernel: k_edge<ST, MODE, ...> / k_edge_mask<ST, MODE, ...> (MODE 0 fwd,
    1 dst pass, 2 src pass); None for other kernels."""
    if short.startswith("k_edge_mask_dual<"):
        return "sir_edge_agg_bwd"
    for pre in ("k_edge_mask<", "k_edge<"):
        if short.startswith(pre):
            args = short[len(pre):].split(">", 1)[0].split(",")
            try:
                return PASSES[int(args[1])]
            except (IndexError, ValueError, KeyError):
                return None
    return None


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            key = (r.get("Agent_Id", ""), int(r["Dispatch_Id"]))
            name = r["Kernel_Name"]
            per.setdefault(key, [name, 0.0])
            per[key][1] += float(r["Counter_Value"])
    return [per[k] for k in sorted(per, key=lambda k: k[1])]


def by_pass(rows):
    out = defaultdict(list)
    cur = None
    for name, val in rows:
        short = name.split("sir::", 1)[-1] if "sir::" in name else name
        hit = pass_of(short)
        if hit is not None:
            cur = [hit, val]
            out[hit].append(cur)
        elif short.startswith("k_combine") and cur is not None:
            cur[1] += val
        else:
            cur = None
    return {k: [v for _, v in lst] for k, lst in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--graph", default="S2")
    ap.add_argument("--agg", default="sum")
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16", "f16"])
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fetch = by_pass(load(a.fetch_dir, "FETCH_SIZE"))
    write = by_pass(load(a.write_dir, "WRITE_SIZE"))
    res = {"graph": a.graph, "agg": a.agg, "H": a.H, "dtype": a.dtype,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; bytes = "
                     "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per launch (gfx950 FETCH_SIZE half-count "
                     "correction for 16 B/lane reads); median over launches"
                     + ("" if a.dtype == "f32" else "; 16-bit storage gathers 8 B per lane, a width the x2 "
                        "correction is not calibrated for (MI355X_MICROARCH.md): fetch bytes are an upper "
                        "bound, fetch_kib_raw the lower one"),
           "build": build_id(),
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = sorted(fetch.get(k, [0.0]))
        w = sorted(write.get(k, [0.0]))
        fm, wm = f[len(f) // 2], w[len(w) // 2]
        res["kernels"][k] = {"fetch_kib": fm, "fetch_kib_raw": fm, "write_kib": wm, "launches": len(f),
                             "hbm_bytes_per_launch": int(2 * fm * 1024 + wm * 1024)}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

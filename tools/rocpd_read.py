#!/usr/bin/env python3
"""Summarise a rocprofv3 run_results.db: per kernel (substring filter) the launch count, mean
duration and the mean of every PMC counter collected.  python tools/rocpd_read.py DB [--match gemm]"""
import argparse
import collections
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db", nargs="+")
ap.add_argument("--match", default="")
a = ap.parse_args()
for f in a.db:
    c = sqlite3.connect(f)
    names = {i: n for i, n in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    disp = list(c.execute("select id, kernel_id, start, end from rocpd_kernel_dispatch"))
    pmc = collections.defaultdict(dict)
    try:
        pn = {i: n for i, n in c.execute("select id, name from rocpd_info_pmc")}
        ecol = [r[1] for r in c.execute("pragma table_info(rocpd_pmc_event)")]
        for row in c.execute("select * from rocpd_pmc_event"):
            d = dict(zip(ecol, row))
            key = d.get("event_id")
            pmc[key][pn[d["pmc_id"]]] = pmc[key].get(pn[d["pmc_id"]], 0) + d["value"]
        ev = {r[0]: r[1] for r in c.execute("select id, correlation_id from rocpd_event")} if pmc else {}
    except sqlite3.Error:
        pass
    agg = collections.defaultdict(lambda: {"n": 0, "ms": 0.0, "pmc": collections.Counter()})
    dispatch_events = {}
    try:
        dcol = [r[1] for r in c.execute("pragma table_info(rocpd_kernel_dispatch)")]
        for row in c.execute("select * from rocpd_kernel_dispatch"):
            d = dict(zip(dcol, row))
            dispatch_events[d["id"]] = d.get("event_id")
    except sqlite3.Error:
        pass
    for i, kid, s, e in disp:
        n = names.get(kid, "?")
        if a.match not in n:
            continue
        g = agg[n]
        g["n"] += 1
        g["ms"] += (e - s) / 1e6
        evid = dispatch_events.get(i)
        for k, v in pmc.get(evid, {}).items():
            g["pmc"][k] += v
    print(f)
    for n, g in agg.items():
        line = f"  {g['n']:3d} x {g['ms'] / g['n']:8.3f} ms  {n[:90]}"
        print(line)
        for k, v in sorted(g["pmc"].items()):
            print(f"        {k:28s} {v / g['n']:.4g}")

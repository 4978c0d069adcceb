#!/usr/bin/env python3
"""rocprofv3 --stats kernel_stats.csv -> a short table (calls, avg ms, share, name cut to 110 chars).

    python tools/kernel_summary.py gpurun_out/final/S2/prof/run_kernel_stats.csv --title "..." > profiles/r02_S2_kernel_summary.txt
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    if a.title:
        print(f"# {a.title}")
    print(f"{'calls':>6} {'avg_ms':>9} {'total%':>7}  kernel")
    for r in rows[:a.top]:
        name = r["Name"]
        name = name if len(name) <= 110 else name[:107] + "..."
        print(f"{int(r['Calls']):6d} {float(r['AverageNs']) / 1e6:9.3f} {float(r['Percentage']):7.2f}  {name}")


if __name__ == "__main__":
    main()

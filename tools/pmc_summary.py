#!/usr/bin/env python3
"""Per-kernel means of every counter in a directory of rocprofv3 --pmc passes.

    python tools/pmc_summary.py gpurun_out/pmcg [--match gemm]
Each sub-directory is one pass (<shape>_p<i>); counters are summed over a dispatch's per-XCD/SE
rows and averaged over the dispatches of a kernel.  Derived ratios (per-SIMD MFMA busy, wait
shares) are printed when their inputs are present."""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    groups = defaultdict(lambda: defaultdict(list))     # (prefix, kernel) -> counter -> values
    for sub in sorted(glob.glob(os.path.join(a.dir, "*"))):
        if not os.path.isdir(sub):
            continue
        prefix = re.sub(r"_p\d+$", "", os.path.basename(sub))
        for f in glob.glob(os.path.join(sub, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            names = {}
            for r in csv.DictReader(open(f)):
                key = (int(r["Dispatch_Id"]), r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
            for (d, c), v in per.items():
                k = names[d]
                k = k.replace("(anonymous namespace)::", "")
                short = k.split("sir::", 1)[-1] if "sir::" in k else k
                short = re.sub(r"\(.*", "", short)[:80]
                if a.match and a.match not in short:
                    continue
                groups[(prefix, short)][c].append(v)
    for (prefix, k), cs in sorted(groups.items()):
        print(f"== {prefix}  {k}")
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        for c in sorted(m):
            print(f"   {c:32s} {m[c]:16.4g}  (n={len(cs[c])})")
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"] > 0:
            wc = m["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"   share {c:26s} {m[c] / wc:8.3f} of wave cycles")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m and m["GRBM_GUI_ACTIVE"] > 0:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs
            print(f"   MFMA busy per SIMD            {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8) / 1024:8.3f}")


if __name__ == "__main__":
    main()

#!/bin/bash
# round-6 call 9: the split dz pass (each edge's entries over both half-waves) A/B + kernel times
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b9
mkdir -p $O
timeout -k 10 300 python -u tools/maxsrcord_ab.py --env SIR_MAXB_SPLIT --forms 0,1,2 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/maxsrcord_ab.py --env SIR_MAXB_SPLIT --rounds 2 --forms 2,0 > $O/prof.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) --top 10 > $O/summary.txt
cat $O/summary.txt

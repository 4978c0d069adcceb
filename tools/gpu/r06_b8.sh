#!/bin/bash
# round-6 call 8: max backward with the dK pass on source-ordered entries (A/B, bit-identity) + kernel times
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b8
mkdir -p $O
timeout -k 10 300 python -u tools/maxsrcord_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
export SIR_MAXB_SRCORD=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/maxsrcord_ab.py --rounds 3 --forms 1 > $O/prof.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) --top 14 > $O/summary.txt
cat $O/summary.txt

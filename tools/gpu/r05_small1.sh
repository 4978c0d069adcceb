#!/bin/bash
# round-5: per-launch times of the config-5 GEMMs (eager / graph) and a cfg5 rocprof of the probe
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_small1
mkdir -p $O
timeout -k 10 300 python -u tools/dbg/small_gemm_probe.py > $O/probe.txt 2>&1; rc=$?
cat $O/probe.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/dbg/small_gemm_probe.py > $O/prof.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) --top 20 > $O/summary.txt
cat $O/summary.txt

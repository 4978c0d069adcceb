#!/bin/bash
# round-5: cfg5 step kernel profile inside the replayed HIP graph
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_cfg5prof; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload ${WL:-cfg5} --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/prof.log 2>&1 || exit $?
f=$(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/kernel_summary.py $f --top 40 > $O/summary.txt
cat $O/summary.txt
tail -1 $O/prof.log | cut -c1-300

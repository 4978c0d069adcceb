#!/bin/bash
# round-6 call 6: S1 max step in f32 and bf16 (the 16-bit max forward) with rocprof kernel summaries
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b6
mkdir -p $O
for d in f32 bf16; do
  timeout -k 10 400 python -u bench.py --graph S1 --agg max --dtype $d --steps 10 --warmup 3 --no-cpu-baseline --no-aux > $O/b_S1max_$d.json 2> $O/b_S1max_$d.err || { tail -5 $O/b_S1max_$d.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_S1max_$d.json')); print('S1max $d', d['ms_per_step'], d.get('ms_per_step_median'))"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$d -o run --output-format csv -- python3 bench.py --graph S1 --agg max --dtype $d --steps 3 --warmup 1 --no-cpu-baseline --no-aux > $O/prof_$d.log 2>&1 || exit $?
  python3 tools/kernel_summary.py $(ls $O/prof_$d/*/run_kernel_stats.csv $O/prof_$d/run_kernel_stats.csv 2>/dev/null | head -1) --top 16 > $O/S1max_${d}_summary.txt
  cat $O/S1max_${d}_summary.txt
done

#!/bin/bash
# round-4 final set B: the other bench lines, rocprof summaries of S1 max / cfg1 / cfg2 / cfg5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final4
mkdir -p $O
for a in "S1:--graph S1" "S2mean:--agg mean" "S2sym:--agg sym" "S1max:--graph S1 --agg max" "cfg1:--workload cfg1" "cfg2:--workload cfg2" "cfg3:--workload cfg3" "cfg5:--workload cfg5"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 400 python -u bench.py $x --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'), d.get('roofline', {}).get('frac'))"
done
for a in "S1max:--graph S1 --agg max" "cfg1:--workload cfg1" "cfg2:--workload cfg2" "cfg5:--workload cfg5"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 bench.py $x --steps 5 --warmup 2 --no-cpu-baseline --no-aux --no-capture > $O/prof_$n.log 2>&1 || exit $?
  python3 tools/kernel_summary.py $(ls $O/prof_$n/*/run_kernel_stats.csv $O/prof_$n/run_kernel_stats.csv 2>/dev/null | head -1) --top 20 > $O/${n}_summary.txt
  head -12 $O/${n}_summary.txt
done

#!/bin/bash
# round 4: cfg1 / cfg5 / S1 max bench lines + rocprof kernel summaries (hipBLASLt Cijk_* kernels must be gone)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
for a in "cfg1:--workload cfg1" "cfg5:--workload cfg5" "S1max:--graph S1 --agg max" "cfg2:--workload cfg2"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 300 python -u bench.py $x --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'), d.get('roofline', {}).get('frac'))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 bench.py $x --steps 5 --warmup 2 --no-cpu-baseline --no-aux --no-capture > $O/prof_$n.log 2>&1 || exit $?
  python3 tools/kernel_summary.py $(ls $O/prof_$n/*/run_kernel_stats.csv $O/prof_$n/run_kernel_stats.csv 2>/dev/null | head -1) --top 20 > $O/${n}_summary.txt
  head -24 $O/${n}_summary.txt
done

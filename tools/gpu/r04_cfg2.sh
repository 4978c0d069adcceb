#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
for a in "cfg2:--workload cfg2" "cfg5:--workload cfg5" "cfg1:--workload cfg1"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 300 python -u bench.py $x --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg2 -o run --output-format csv -- python3 bench.py --workload cfg2 --steps 5 --warmup 2 --no-cpu-baseline --no-aux --no-capture > $O/prof_cfg2.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof_cfg2/*/run_kernel_stats.csv $O/prof_cfg2/run_kernel_stats.csv 2>/dev/null | head -1) --top 24 > $O/cfg2_summary.txt
cat $O/cfg2_summary.txt

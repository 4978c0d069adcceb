#!/bin/bash
# round-5: max backward over destination-row ranges (the S2 shape) — the edge-MLP GPU tests, the S2 / S1 max lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_max1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for a in "S2max:--graph S2 --agg max" "S1max:--graph S1 --agg max"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 600 python -u bench.py $x --steps 10 --warmup 3 --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'), d.get('value'))"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_S2max -o run --output-format csv -- python3 bench.py --graph S2 --agg max --steps 3 --warmup 1 --no-cpu-baseline --no-aux --no-capture > $O/prof_S2max.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof_S2max/*/run_kernel_stats.csv $O/prof_S2max/run_kernel_stats.csv 2>/dev/null | head -1) --top 20 > $O/S2max_summary.txt
head -22 $O/S2max_summary.txt

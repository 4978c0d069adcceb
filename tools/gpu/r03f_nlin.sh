# native nn.Linear for the edge-MLP / max / modular projections: GPU suite, cfg1 and S1 max lines
set -o pipefail
O=gpurun_out/nlin
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
for a in "cfg1:--workload cfg1" "S1max:--graph S1 --agg max"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 400 python -u bench.py $x --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cfg1 -o run --output-format csv -- python3 bench.py --workload cfg1 --steps 6 --warmup 2 --no-capture --no-cpu-baseline --no-aux > $O/cfg1.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/cfg1/*/run_kernel_stats.csv $O/cfg1/run_kernel_stats.csv 2>/dev/null | head -1) --top 20 > $O/cfg1_summary.txt; cat $O/cfg1_summary.txt

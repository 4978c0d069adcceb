# round-3 final build: GPU suite, smoke, the default bench line + rocprof kernel summary of the S2 step, the other lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/b_S2.json 2> $O/b_S2.err || exit $?
python3 -c "import json; d=json.load(open('$O/b_S2.json')); print('S2', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['frac'], d['projections']['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/prof.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) --top 16 > $O/S2_summary.txt; cat $O/S2_summary.txt
for a in "S2bf16:--dtype bf16" "S1:--graph S1" "S2mean:--agg mean" "S2sym:--agg sym" "S1max:--graph S1 --agg max" "cfg1:--workload cfg1" "cfg2:--workload cfg2" "cfg3:--workload cfg3" "cfg3nodrop:--workload cfg3 --dropout 0" "cfg5:--workload cfg5"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 400 python -u bench.py $x --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'), d.get('roofline', {}).get('frac'))"
done

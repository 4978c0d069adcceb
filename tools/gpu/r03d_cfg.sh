# small-batch stack workloads: GraphNorm + stack tests, bench lines and rocprof kernel stats of cfg5 / cfg1
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cfg
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_stacks_gpu.py tests/test_gpu_parity.py -x -q -k "graph_norm or graphnorm or stack or cfg" --timeout 200 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
for w in cfg5 cfg1 cfg3 cfg2; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$w.json 2> $O/b_$w.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$w.json')); print('$w', d['ms_per_step'], d.get('ms_per_step_median'))"
done
for w in cfg5 cfg1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-aux --no-capture > $O/prof_$w.log 2>&1 || exit $?
  python3 tools/kernel_summary.py $O/prof_$w/run_kernel_stats.csv --top 30
done

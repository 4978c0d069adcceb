# cfg5 with the native small-batch GEMM route vs torch's (SIRGCN_GEMM_MIN_ROWS), same box; rocprof of the native route
set -o pipefail
O=gpurun_out/cfg5n
mkdir -p $O
for mr in 0 32768 0 32768; do
  SIRGCN_GEMM_MIN_ROWS=$mr timeout -k 10 300 python -u bench.py --workload cfg5 --steps 30 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$mr.json 2> $O/b_$mr.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$mr.json')); print('cfg5 min_rows=$mr', d['ms_per_step'], d.get('ms_per_step_median'))"
done
SIRGCN_GEMM_MIN_ROWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 10 --warmup 2 --no-capture --no-cpu-baseline --no-aux > $O/prof.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) --top 30

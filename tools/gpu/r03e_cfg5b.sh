# small-batch route v2 (direct-weight NT, 4-wave split-k tiles; 4-wave TN): GEMM tests, cfg5 / cfg1 native vs torch
# route on one box, rocprof of cfg5 native, then the GPU suite
set -o pipefail
O=gpurun_out/cfg5b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -4 $O/tests.log; [ $r -eq 0 ] || exit $r
for w in cfg5 cfg1; do
for mr in 0 32768 0 32768; do
  SIRGCN_GEMM_MIN_ROWS=$mr timeout -k 10 300 python -u bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline --no-aux > $O/b_${w}_$mr.json 2> $O/b_${w}_$mr.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_${w}_$mr.json')); print('$w min_rows=$mr', d['ms_per_step'], d.get('ms_per_step_median'))"
done
done
SIRGCN_GEMM_MIN_ROWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 10 --warmup 2 --no-capture --no-cpu-baseline --no-aux > $O/prof.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) --top 24 > $O/summary.txt; cat $O/summary.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1; r=$?; tail -3 $O/suite.log; exit $r

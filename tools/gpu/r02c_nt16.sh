# 16-bit NT GEMM for the autocast layer: numerics tests, autocast layer/stack tests, then S2 bf16 and
# cfg2 bench lines and a rocprof kernel summary of the bf16 step.
set -o pipefail
mkdir -p gpurun_out/nt16
O=gpurun_out/nt16
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_amp_gpu.py tests/test_stacks_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u bench.py --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_S2bf16.json 2> $O/b_S2bf16.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_S2bf16.json
timeout -k 10 300 python -u bench.py --workload cfg2 --steps 20 --warmup 5 > $O/b_cfg2.json 2> $O/b_cfg2.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_cfg2.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/prof.log 2>&1 || exit $?
f=$(ls $O/prof/*kernel_stats.csv | head -1); python3 tools/kernel_summary.py $f --top 16 > $O/summary.txt; cat $O/summary.txt

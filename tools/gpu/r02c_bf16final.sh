# after the 16-bit dK unroll change: whole GPU suite, then the bf16 S2 and cfg2 bench lines
set -o pipefail
mkdir -p gpurun_out/bf16f
O=gpurun_out/bf16f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -2 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u bench.py --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_S2bf16.json 2> $O/b_S2bf16.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_S2bf16.json | head -1
timeout -k 10 300 python -u bench.py --workload cfg2 --steps 20 --warmup 5 > $O/b_cfg2.json 2> $O/b_cfg2.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_cfg2.json | head -1

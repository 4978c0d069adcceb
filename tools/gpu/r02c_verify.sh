# Re-entry check of HEAD on a fresh box: the whole -m gpu suite, then S2 fp32 / bf16 bench lines.
set -o pipefail
mkdir -p gpurun_out/verify
O=gpurun_out/verify
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -5 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_S2.json 2> $O/b_S2.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_S2.json
timeout -k 10 300 python -u bench.py --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_S2bf16.json 2> $O/b_S2bf16.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_S2bf16.json

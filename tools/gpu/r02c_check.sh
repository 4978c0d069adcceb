# GEMM + parity + AMP + stack tests, then S2 f32 / bf16 and cfg2 / cfg3 bench lines
set -o pipefail
mkdir -p gpurun_out/chk
O=gpurun_out/chk
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -2 $O/tests.log; [ $r -eq 0 ] || exit $r
for a in "S2:" "S2bf16:--dtype bf16" "cfg2:--workload cfg2" "cfg3:--workload cfg3"; do n=${a%%:*}; x=${a#*:}; timeout -k 10 300 python -u bench.py $x --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || exit $?; echo "$n $(grep -o '"ms_per_step": [0-9.]*' $O/b_$n.json | head -1)"; done

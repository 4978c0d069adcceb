# final build check: smoke, whole GPU suite, S2 headline line (with cpu_baseline) and S1
set -o pipefail
mkdir -p gpurun_out/last
O=gpurun_out/last
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; r=$?; tail -1 $O/smoke.log; [ $r -eq 0 ] || exit $r
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -2 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > $O/b_S2.json 2> $O/b_S2.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_S2.json | head -1
timeout -k 10 300 python -u bench.py --graph S1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b_S1.json 2> $O/b_S1.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_S1.json | head -1

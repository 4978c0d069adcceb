# round-3 measurement set, part A: GPU suite, smoke, the default bench line, rocprof + PMC of the S2 step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/finalA
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_S2.json 2> $O/bench_S2.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_S2.json')); print('S2', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['frac'], d['projections']['ms_per_step'])"
BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-aux" bash tools/profile_round.sh $O/S2 || exit $?
python3 tools/kernel_summary.py $O/S2/prof/run_kernel_stats.csv --top 16

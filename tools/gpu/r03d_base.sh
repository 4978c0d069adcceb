# session-4 baseline: GPU suite + smoke, default bench line, rocprof kernel stats of the S2 step,
# and the stand-alone GEMM shapes
set -o pipefail
O=gpurun_out/base
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -6 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d.get('ms_per_step_median'), d['projections']['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/prof.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/gemm_bench.py > $O/gemm.log 2>&1 || exit $?
cat $O/gemm.log

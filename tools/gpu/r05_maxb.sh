#!/bin/bash
# routed max backward: GPU tests, then S1 max / S2 max lines and a rocprof summary of S1 max
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/maxb
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_edgemlp_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
line() { n=$1; shift; timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-aux "$@" > $O/b_$n.json 2> $O/b_$n.err || { tail -20 $O/b_$n.err; exit 1; }; python3 -c "import json;d=json.load(open('$O/b_$n.json'));print('$n',d['ms_per_step'],d.get('ms_per_step_median'))"; }
line S1max --graph S1 --agg max --steps 10 --warmup 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_S1max -o run --output-format csv -- python3 bench.py --graph S1 --agg max --steps 3 --warmup 1 --no-cpu-baseline --no-aux > $O/prof_S1max.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof_S1max/*/run_kernel_stats.csv $O/prof_S1max/run_kernel_stats.csv 2>/dev/null | head -1) --top 20 > $O/S1max_summary.txt
cat $O/S1max_summary.txt
line S2max --graph S2 --agg max --steps 5 --warmup 2

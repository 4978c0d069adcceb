#!/bin/bash
# round-6 call 7: the autocast projections on the native 16-bit GEMMs (linalg._Linear16):
# AMP tests, then the S1 max bf16 step with its rocprof kernel summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b7
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_amp_gpu.py tests/test_edgemlp_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
d=bf16
timeout -k 10 400 python -u bench.py --graph S1 --agg max --dtype $d --steps 10 --warmup 3 --no-cpu-baseline --no-aux > $O/b_S1max_$d.json 2> $O/b_S1max_$d.err || { tail -5 $O/b_S1max_$d.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_S1max_$d.json')); print('S1max $d', d['ms_per_step'], d.get('ms_per_step_median'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$d -o run --output-format csv -- python3 bench.py --graph S1 --agg max --dtype $d --steps 3 --warmup 1 --no-cpu-baseline --no-aux > $O/prof_$d.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof_$d/*/run_kernel_stats.csv $O/prof_$d/run_kernel_stats.csv 2>/dev/null | head -1) --top 20 > $O/S1max_${d}_summary.txt
cat $O/S1max_${d}_summary.txt

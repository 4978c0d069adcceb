#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_onehot; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
SIRGCN_MAX_ONEHOT=$v timeout -k 10 400 python -u bench.py --graph S1 --agg max --steps 10 --warmup 3 --no-cpu-baseline --no-aux > $O/b_S1max_$v.json 2> $O/b_S1max_$v.err || { tail -5 $O/b_S1max_$v.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_S1max_$v.json')); print('S1max onehot=$v', d['ms_per_step'], d.get('ms_per_step_median'))"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --graph S1 --agg max --steps 3 --warmup 1 --no-cpu-baseline --no-aux > $O/prof.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) --top 14 > $O/summary.txt; cat $O/summary.txt

#!/bin/bash
# round-6 call 19: max / dist tests on the route-cap build; cfg3 kernel summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b19
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_gpu.py tests/test_dist_gpu.py tests/test_amp_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload cfg3 --steps 10 --warmup 3 --no-cpu-baseline --no-aux --no-capture > $O/prof.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) --top 24 > $O/cfg3_summary.txt; cat $O/cfg3_summary.txt

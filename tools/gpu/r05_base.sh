#!/bin/bash
# round-5: GPU tests touched by this round's edits (edge-MLP max incl. negative slope, GEMMs, dropout, edge-cut
# incl. max and range-chunked parts, the 8-rank S2 edge-cut) + the S2 max bench line with its rocprof summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_base
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_edgemlp_gpu.py tests/test_gemm_gpu.py tests/test_dropout_gpu.py tests/test_dist_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_cfg4_gpu.py -m gpu -x -q -k "8_ranks" --timeout 600 --timeout-method thread > $O/pytest_cfg4.log 2>&1; rc=$?
tail -3 $O/pytest_cfg4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --graph S2 --agg max --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/b_S2max.json 2> $O/b_S2max.err || { tail -5 $O/b_S2max.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_S2max.json')); print('S2max', d['ms_per_step'], d.get('ms_per_step_median'), d.get('value'))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_S2max -o run --output-format csv -- python3 bench.py --graph S2 --agg max --steps 3 --warmup 1 --no-cpu-baseline --no-aux --no-capture > $O/prof_S2max.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof_S2max/*/run_kernel_stats.csv $O/prof_S2max/run_kernel_stats.csv 2>/dev/null | head -1) --top 20 > $O/S2max_summary.txt
head -16 $O/S2max_summary.txt

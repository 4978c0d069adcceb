#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_gn2; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "graph_norm" -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest1.log 2>&1; rc=$?
tail -2 $O/pytest1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_stacks_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest2.log 2>&1; rc=$?
tail -4 $O/pytest2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 50 --warmup 10 --no-cpu-baseline --no-aux > $O/b_cfg5.json 2> $O/b_cfg5.err || { tail -5 $O/b_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_cfg5.json')); print('cfg5', d['ms_per_step'], d.get('ms_per_step_median'))"

#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_gn; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "graph_norm" tests/test_stacks_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for a in "64 25 300" "64 60 300" "10000 23 128"; do timeout -k 10 60 ./tools/dbg/gn_probe $a || exit 1; done
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 50 --warmup 10 --no-cpu-baseline --no-aux > $O/b_cfg5.json 2> $O/b_cfg5.err || { tail -5 $O/b_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_cfg5.json')); print('cfg5', d['ms_per_step'], d.get('ms_per_step_median'))"

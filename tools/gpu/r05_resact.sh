#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_resact; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stacks_gpu.py tests/test_amp_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in cfg2 cfg3 cfg5; do
timeout -k 10 300 python -u bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$w.json 2> $O/b_$w.err || { tail -5 $O/b_$w.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_$w.json')); print('$w', d['ms_per_step'], d.get('ms_per_step_median'))"
done

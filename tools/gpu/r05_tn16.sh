#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_tn16; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -k "tn16" -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
SIR_TN16_NARROW=$v timeout -k 10 300 python -u bench.py --workload cfg2 --steps 30 --warmup 5 --no-cpu-baseline --no-aux > $O/b_cfg2_$v.json 2> $O/b_cfg2_$v.err || { tail -5 $O/b_cfg2_$v.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_cfg2_$v.json')); print('cfg2 narrow=$v', d['ms_per_step'], d.get('ms_per_step_median'))"
done

#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_nt16; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -k "nt16" tests/test_amp_gpu.py tests/test_stacks_gpu.py tests/test_dropout_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
SIR_NT16_NARROW=$v timeout -k 10 300 python -u bench.py --workload cfg2 --steps 30 --warmup 5 --no-cpu-baseline --no-aux > $O/b_cfg2_$v.json 2> $O/b_cfg2_$v.err || { tail -5 $O/b_cfg2_$v.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_cfg2_$v.json')); print('cfg2 nt16 narrow=$v', d['ms_per_step'], d.get('ms_per_step_median'))"
done
for w in cfg5 cfg3; do
timeout -k 10 300 python -u bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline --no-aux > $O/b_$w.json 2> $O/b_$w.err || { tail -5 $O/b_$w.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_$w.json')); print('$w', d['ms_per_step'], d.get('ms_per_step_median'))"
done

#!/bin/bash
# round-5: small-batch route — LT kernels + side-stream weight gradients: tests, cfg5 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_small3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py "tests/test_gpu_parity.py::test_weight_grads_on_side_stream_bit_identical" -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
run() { n=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --workload cfg5 --steps 50 --warmup 10 --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'))"; }
run base SIR_LT_NT=0 SIR_LT_TN=0 SIRGCN_OVERLAP_ROWS=0
run lt SIRGCN_OVERLAP_ROWS=0
run ov SIR_LT_NT=0 SIR_LT_TN=0
run lt_ov X=1
run lt_ov_nt2 SIR_LT_NT=2

#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_w8; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
LT_CFGS=2,3,6,7,8,4,5 timeout -k 10 300 python -u tools/dbg/small_gemm_probe.py > $O/probe.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/probe.txt | grep -v "torch\."

#!/bin/bash
# round-5: LDS-tiled small GEMM (k_gemm_lt) — GEMM GPU tests, then the per-arrangement probe
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_small2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dbg/small_gemm_probe.py > $O/probe.txt 2>&1; rc=$?
cat $O/probe.txt
exit $rc

#!/bin/bash
# round-6 call 1: the NT GEMM VALU-trim A/B, the max dW_R kernel A/B, then the advisor-fix GPU tests + smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b1
mkdir -p $O
O=$O tools/gpu/r06_gemm_ab.sh || exit $?
timeout -k 10 300 python -u tools/maxdw_ab.py > $O/maxdw_ab.txt 2>&1 || exit $?
cat $O/maxdw_ab.txt
O=$O tools/gpu/r06_advice.sh

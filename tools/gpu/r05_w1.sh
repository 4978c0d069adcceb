#!/bin/bash
# round-5: wave-specialised NT GEMM (k_gemm_nt_w) vs k_gemm_nt_p on the S2 shapes, and the GEMM tests on the w route
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_w1
mkdir -p $O
L=sir-gcn_amd/lib/libsirconv.so
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 5 --only QK,Y,G,dX --libs p=$L w=$L@SIR_GEMM_NT_ROUTE=w > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
SIR_GEMM_NT_ROUTE=w timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
exit $rc

#!/bin/bash
# round-6 call 3: k_max_dw_qk2 branch-free accumulation at 2 blocks / CU (128 VGPRs) vs 1 block / CU, vs k_max_dw_qk
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b3
mkdir -p $O
timeout -k 10 300 python -u tools/maxdw_ab.py --forms 1,2,2@occ1 --libs occ1=sir-gcn_amd/lib/libsirconv_occ1.so > $O/maxdw_ab.txt 2>&1; rc=$?
cat $O/maxdw_ab.txt
exit $rc

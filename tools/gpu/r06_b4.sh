#!/bin/bash
# round-6 call 4: k_max_dw_qk2 with Q rows staged in LDS two batches ahead (fewer VGPRs) vs k_max_dw_qk; max tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b4
mkdir -p $O
timeout -k 10 300 python -u tools/maxdw_ab.py --forms 1,2 > $O/maxdw_ab.txt 2>&1 || { cat $O/maxdw_ab.txt; exit 1; }
cat $O/maxdw_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
exit $rc

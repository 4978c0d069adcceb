#!/bin/bash
# round-6 call 5: k_max_dw_qk2 (Q rows staged in LDS) A/B; the 16-bit max forward tests; max / AMP suites
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b5
mkdir -p $O
timeout -k 10 300 python -u tools/maxdw_ab.py --forms 1,2 > $O/maxdw_ab.txt 2>&1 || { cat $O/maxdw_ab.txt; exit 1; }
cat $O/maxdw_ab.txt
timeout -k 10 900 python -u -m pytest tests/test_amp_gpu.py tests/test_edgemlp_gpu.py -m gpu -q -x --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert" $O/tests.log | tail -15
exit $rc

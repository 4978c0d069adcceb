#!/bin/bash
# round-5: the whole GPU test suite (one process, per-test timeout)
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/final5}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1; rc=$?
tail -15 $O/suite.log
exit $rc

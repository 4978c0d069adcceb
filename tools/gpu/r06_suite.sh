#!/bin/bash
# round-6: the whole -m gpu suite on the shipped build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final6
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
rc=$?
tail -45 $O/suite.log
exit $rc

#!/bin/bash
# round-6: smoke + the whole -m gpu suite on the final build
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/final6b}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/suite.log | tail -3
exit $rc

#!/bin/bash
# round 4: smoke + GPU suite (one process), log under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r04_smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest ${SUITE:-tests} -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/r04_suite.log 2>&1
rc=$?
echo "suite rc $rc"
grep -E "passed|failed|FAILED|Error" gpurun_out/r04_suite.log | tail -30
exit $rc

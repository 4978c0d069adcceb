#!/bin/bash
# round-6: the GPU tests touched by the advisor fixes (empty-graph max backward partials, pair-GEMM
# fallback off the LDS kernel, hashed per-rank dropout on the edge-cut max path) + smoke
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r06a}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests/test_edgemlp_gpu.py tests/test_gemm_gpu.py tests/test_dist_gpu.py -m gpu -q -x \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
exit $rc

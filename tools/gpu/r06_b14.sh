#!/bin/bash
# round-6 call 14: dW_R (k_max_dw_qk2) with batch-local arg offsets staged (no row-bound reads or branches
# in the accumulation loop) vs the previous build; S1 max shape, bit-identity; then the max tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b14
mkdir -p $O
timeout -k 10 300 python -u tools/maxdw_ab.py --forms 2,2@base --libs base=sir-gcn_amd/lib/libsirconv_base.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_gpu.py tests/test_amp_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log

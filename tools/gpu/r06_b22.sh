#!/bin/bash
# round-6 call 22: stream max forward staging split by v_fma_mix (mix1, shipped) vs the C split (mix0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b22
mkdir -p $O
timeout -k 10 300 python -u tools/mlpfwd_ab.py --libs mix1=sir-gcn_amd/lib/libsirconv.so mix0=sir-gcn_amd/lib/libsirconv_mix0.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log

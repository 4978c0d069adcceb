#!/bin/bash
# round-6 call 11: the routed dz passes on a work queue (ABI 16) vs the static item assignment (the
# previous build, libsirconv_static.so): max backward A/B on S1 / S2 (bit-identity), then the max tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b11
mkdir -p $O
for gr in S1 S2; do
  r=7; [ $gr = S2 ] && r=4
  timeout -k 10 400 python -u tools/maxbwd_ab.py --graph $gr --rounds $r --libs queue=sir-gcn_amd/lib/libsirconv.so static=sir-gcn_amd/lib/libsirconv_static.so > $O/ab_$gr.txt 2>&1 || { tail -20 $O/ab_$gr.txt; exit 1; }
  grep -v amdgpu.ids $O/ab_$gr.txt
done
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_gpu.py tests/test_amp_gpu.py tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log

#!/bin/bash
# round-6 call 26: stream max forward with interior tiles walked by both half-waves (walk1, shipped) vs the
# one-half walk (walk0): A/B f32 + bf16 (bit-identity), edge-MLP + AMP tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b26
mkdir -p $O
for d in f32 bf16; do
  timeout -k 10 300 python -u tools/mlpfwd_ab.py --dtype $d --libs walk1=sir-gcn_amd/lib/libsirconv.so walk0=sir-gcn_amd/lib/libsirconv_walk0.so > $O/ab_$d.txt 2>&1 || { tail -20 $O/ab_$d.txt; exit 1; }
  grep -v amdgpu.ids $O/ab_$d.txt
done
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_gpu.py tests/test_amp_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log

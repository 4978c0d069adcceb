#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for g in sym sum; do
timeout -k 10 500 python tools/edge_ab.py --graph S2 --agg $g --libs new=sir-gcn_amd/lib/libsirconv.so prev=sir-gcn_amd/lib/libsirconv_prev.so nods=sir-gcn_amd/lib/libsirconv_nods.so 2>&1 | grep -v amdgpu | sed "s/^/$g /" || exit 1
done 2>&1 | tee gpurun_out/r04_ab_devseed.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dropout_gpu.py tests/test_gpu_parity.py 2>&1 | tail -2

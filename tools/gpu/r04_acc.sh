#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/edge_ab.py --graph S2 --libs new=sir-gcn_amd/lib/libsirconv.so acc=sir-gcn_amd/lib/libsirconv_acc.so 2>&1 | tee gpurun_out/r04_ab_acc.txt &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_dist_gpu.py tests/test_small_width_gpu.py 2>&1 | tail -3

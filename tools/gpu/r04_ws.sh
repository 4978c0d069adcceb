#!/bin/bash
# Weight-stationary NT GEMM (k_gemm_nt_ws) vs the persistent k_gemm_nt_p: interleaved A/B on the
# S2 projection shapes (d = 0 means bit-identical to the first library), then the GEMM tests.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/gemm_ab.py --rounds 7 --only QK,Y,G,dX \
    --libs p=sir-gcn_amd/lib/libsirconv.so ws=sir-gcn_amd/lib/libsirconv_ws.so ns3=sir-gcn_amd/lib/libsirconv_ns3.so ns4=sir-gcn_amd/lib/libsirconv_ns4.so \
    2>&1 | tee gpurun_out/r04_ab_ws.txt &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_gpu.py -k "nt" \
    2>&1 | tee gpurun_out/r04_ws_tests.txt &&
timeout -k 10 400 python tools/mlp_ab.py --graph S1 --agg max \
    --libs new=sir-gcn_amd/lib/libsirconv.so old=sir-gcn_amd/lib/libsirconv_mlpold.so 2>&1 | tee gpurun_out/r04_ab_mlp.txt &&
timeout -k 10 300 python tools/mlp_ab.py --graph mol --agg sum --H 64 --F 64 \
    --libs new=sir-gcn_amd/lib/libsirconv.so old=sir-gcn_amd/lib/libsirconv_mlpold.so 2>&1 | tee -a gpurun_out/r04_ab_mlp.txt &&
timeout -k 10 300 python tools/mlp_ab.py --graph mol --agg max --H 128 --F 128 \
    --libs new=sir-gcn_amd/lib/libsirconv.so old=sir-gcn_amd/lib/libsirconv_mlpold.so 2>&1 | tee -a gpurun_out/r04_ab_mlp.txt &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_edgemlp_gpu.py \
    2>&1 | tee gpurun_out/r04_mlp_tests.txt

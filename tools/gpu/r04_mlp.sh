#!/bin/bash
# Edge-MLP forward A/B (main library vs the SIR_MLP_PIPE=0 build) + the edge-MLP / GEMM tests.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/mlp_ab.py --graph S1 --agg max \
    --libs new=sir-gcn_amd/lib/libsirconv.so q1=sir-gcn_amd/lib/libsirconv_q1.so old=sir-gcn_amd/lib/libsirconv_mlpold.so 2>&1 | tee gpurun_out/r04_ab_mlp.txt &&
timeout -k 10 300 python tools/mlp_ab.py --graph mol --agg max --H 128 --F 128 \
    --libs new=sir-gcn_amd/lib/libsirconv.so q1=sir-gcn_amd/lib/libsirconv_q1.so old=sir-gcn_amd/lib/libsirconv_mlpold.so 2>&1 | tee -a gpurun_out/r04_ab_mlp.txt &&
timeout -k 10 300 python tools/mlp_ab.py --graph S1 --agg sum --H 256 --F 256 \
    --libs new=sir-gcn_amd/lib/libsirconv.so q1=sir-gcn_amd/lib/libsirconv_q1.so old=sir-gcn_amd/lib/libsirconv_mlpold.so 2>&1 | tee -a gpurun_out/r04_ab_mlp.txt &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_edgemlp_gpu.py \
    tests/test_gemm_gpu.py 2>&1 | tee gpurun_out/r04_mlp_tests.txt | tail -5

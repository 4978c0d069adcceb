#!/bin/bash
# Edge-MLP forward A/B: per-item k_mlp_fwd16q vs the edge-stream k_mlp_fwd16r (same library) + tests
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=sir-gcn_amd/lib/libsirconv.so
timeout -k 10 400 python tools/mlp_ab.py --graph S1 --agg max --libs item=$L stream=$L@stream 2>&1 | tee gpurun_out/r04_ab_mlp.txt &&
timeout -k 10 300 python tools/mlp_ab.py --graph S1 --agg sum --libs item=$L stream=$L@stream 2>&1 | tee -a gpurun_out/r04_ab_mlp.txt &&
timeout -k 10 300 python tools/mlp_ab.py --graph S1 --agg sym --libs item=$L stream=$L@stream 2>&1 | tee -a gpurun_out/r04_ab_mlp.txt &&
timeout -k 10 300 python tools/mlp_ab.py --graph S1 --agg mean --F 40 --libs item=$L stream=$L@stream 2>&1 | tee -a gpurun_out/r04_ab_mlp.txt &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_edgemlp_gpu.py \
    tests/test_gemm_gpu.py tests/test_gpu_parity.py 2>&1 | tee gpurun_out/r04_mlp_tests.txt | tail -5

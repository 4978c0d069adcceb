#!/bin/bash
# VW=8 16-bit sub-wave rows: A/B against the 8-B-lane build (libsirconv_vw4.so), then the 16-bit tests
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 300 python -u tools/edge_ab.py --graph S2 --dtype bf16 --libs vw8=sir-gcn_amd/lib/libsirconv.so vw4=sir-gcn_amd/lib/libsirconv_vw4.so > $O/ab_S2bf16.txt 2>&1 || exit 1
cat $O/ab_S2bf16.txt
timeout -k 10 300 python -u tools/edge_ab.py --graph mol --H 128 --agg sym --dtype bf16 --libs vw8=sir-gcn_amd/lib/libsirconv.so vw4=sir-gcn_amd/lib/libsirconv_vw4.so > $O/ab_molbf16.txt 2>&1 || exit 1
cat $O/ab_molbf16.txt
export SUITE="tests/test_amp_gpu.py tests/test_small_width_gpu.py tests/test_gpu_parity.py tests/test_dist_gpu.py tests/test_dropout_gpu.py"
bash tools/gpu/r04_suite.sh

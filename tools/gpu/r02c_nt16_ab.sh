# 16-bit NT GEMM: LDS-staged whole-row epilogue (libsirconv.so) vs fragment-order stores (epi0); then the GEMM and autocast tests
set -o pipefail
mkdir -p gpurun_out/nt16ab
L=sir-gcn_amd/lib
timeout -k 10 300 python -u tools/gemm16_ab.py --libs epi0=$L/libsirconv_epi0.so epi1=$L/libsirconv.so > gpurun_out/nt16ab/epi.txt 2>&1; r=$?; grep -v amdgpu.ids gpurun_out/nt16ab/epi.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_amp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/nt16ab/tests.log 2>&1; r=$?; tail -2 gpurun_out/nt16ab/tests.log; exit $r

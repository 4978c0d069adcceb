# fp32 persistent NT GEMM: LDS-staged whole-row epilogue (libsirconv.so) vs fragment stores (pepi0); GEMM + layer tests
set -o pipefail
mkdir -p gpurun_out/ntp
L=sir-gcn_amd/lib
timeout -k 10 300 python -u tools/gemm_ab.py --libs pepi0=$L/libsirconv_pepi0.so pepi1=$L/libsirconv.so > gpurun_out/ntp/epi.txt 2>&1; r=$?; grep -v amdgpu.ids gpurun_out/ntp/epi.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ntp/tests.log 2>&1; r=$?; tail -2 gpurun_out/ntp/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > gpurun_out/ntp/b_S2.json 2> gpurun_out/ntp/b_S2.err || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ntp/b_S2.json

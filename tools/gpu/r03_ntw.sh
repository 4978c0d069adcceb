# weight-resident NT GEMM: numerics tests, then A/B against the previous NT kernels on the S2 shapes
set -o pipefail
O=gpurun_out/ntw
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "nt and not nt16" > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 7 --libs old=sir-gcn_amd/lib/libsirconv_ntold.so new=sir-gcn_amd/lib/libsirconv.so > $O/ab.txt 2>&1; r=$?; cat $O/ab.txt; exit $r

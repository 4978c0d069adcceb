set -o pipefail
O=gpurun_out/ntw
mkdir -p $O
L=sir-gcn_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "nt and not nt16" > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u tools/gemm_ab.py --rounds 5 --only QK,Y,dX --libs new=$L/libsirconv.so old=$L/libsirconv_old.so noA=$L/libsirconv_a1.so noAC=$L/libsirconv_a3.so > $O/abl.txt 2>&1; r=$?; cat $O/abl.txt; exit $r

set -o pipefail
O=gpurun_out/ntw
mkdir -p $O
L=sir-gcn_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u tools/gemm_ab.py --rounds 7 --only QK,Y,G,dX --libs new=$L/libsirconv.so old=$L/libsirconv_old.so pd1=$L/libsirconv_pd1.so pd3=$L/libsirconv_pd3.so > $O/pd.txt 2>&1; r=$?; cat $O/pd.txt; exit $r

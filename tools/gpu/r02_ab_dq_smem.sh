set -o pipefail
L=sir-gcn_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=25 -v --timeout 300 --timeout-method thread > gpurun_out/t4.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t4.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/edge_ab.py --graph S2 --rounds 6 --libs base=$L/libsirconv.so nosmem=$L/libsirconv_nosmem.so > gpurun_out/ab4_f32.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/edge_ab.py --graph S2 --rounds 6 --dtype bf16 --libs base=$L/libsirconv.so h4=$L/libsirconv_h4.so h12=$L/libsirconv_h12.so > gpurun_out/ab4_bf16.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/edge_ab.py --graph S2 --rounds 6 --agg mean --libs base=$L/libsirconv.so nosmem=$L/libsirconv_nosmem.so > gpurun_out/ab4_f32_mean.txt 2>&1 || exit $?

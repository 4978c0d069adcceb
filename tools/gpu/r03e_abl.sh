# k_gemm_nt_p time decomposition (timing-only ablations, SIR_ABL_NT bits: 1 loads, 2 stores, 4 split, 8 MFMAs)
# and the random-gather rate by row size (torch kernels)
set -o pipefail
O=gpurun_out/abl
mkdir -p $O
L=sir-gcn_amd/lib
timeout -k 10 300 python -u tools/gather_floor.py > $O/gather.txt 2>&1; r=$?; cat $O/gather.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u tools/gemm_ab.py --rounds 5 --only QK,Y,dX --libs base=$L/libsirconv.so a4=$L/libsirconv_abl4.so a8=$L/libsirconv_abl8.so a3=$L/libsirconv_abl3.so a7=$L/libsirconv_abl7.so a11=$L/libsirconv_abl11.so a15=$L/libsirconv_abl15.so > $O/ab.txt 2>&1; r=$?; cat $O/ab.txt; exit $r

# 16-bit NT GEMM: timing-only ablations (abl1 no A loads, abl2 no C stores, abl3 neither, abl4 no MFMAs) and kc64
set -o pipefail
mkdir -p gpurun_out/nt16ab
L=sir-gcn_amd/lib
timeout -k 10 300 python -u tools/gemm16_ab.py --libs base=$L/libsirconv.so kc64=$L/libsirconv_kc64.so abl1=$L/libsirconv_abl1.so abl2=$L/libsirconv_abl2.so abl3=$L/libsirconv_abl3.so abl4=$L/libsirconv_abl4.so > gpurun_out/nt16ab/abl.txt 2>&1; r=$?; grep -v amdgpu.ids gpurun_out/nt16ab/abl.txt; exit $r

# fp32 TN GEMM timing-only ablation: loads dropped (tnabl) vs base
set -o pipefail
mkdir -p gpurun_out/tnabl
L=sir-gcn_amd/lib
timeout -k 10 300 python -u tools/gemm_ab.py --libs base=$L/libsirconv.so tnabl=$L/libsirconv_tnabl.so > gpurun_out/tnabl/ab.txt 2>&1; r=$?; grep -v amdgpu.ids gpurun_out/tnabl/ab.txt; exit $r

# TN16: split-order reduce with 16 loads in flight (newred) vs one (oldred); row-split minimum 1024 (mr1024, with newred)
set -o pipefail
mkdir -p gpurun_out/tns
L=sir-gcn_amd/lib
timeout -k 10 300 python -u tools/gemm16_ab.py --no-nt --tn 229532,128,128 229532,256,128 2000000,256,256 --libs oldred=$L/libsirconv_oldred.so newred=$L/libsirconv.so mr1024=$L/libsirconv_mr1024.so > gpurun_out/tns/ab.txt 2>&1; r=$?; grep -v amdgpu.ids gpurun_out/tns/ab.txt; exit $r

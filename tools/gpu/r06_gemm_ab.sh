#!/bin/bash
# round-6: VALU trims of the persistent NT GEMM's split (v_max3 row maximum; hi / lo by v_fma_mix in asm
# or as fused C ops), A/B interleaved in one process on the S2 shapes (tools/gemm_ab.py)
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r06g}
mkdir -p $O
L=sir-gcn_amd/lib
timeout -k 10 400 python -u tools/gemm_ab.py --rounds 9 --only QK,Y,G,dX --libs base=$L/libsirconv.so \
  max3=$L/libsirconv_max3.so fma=$L/libsirconv_fma.so mix=$L/libsirconv_mix.so > $O/gemm_ab.txt 2>&1; rc=$?
cat $O/gemm_ab.txt
exit $rc

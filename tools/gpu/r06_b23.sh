#!/bin/bash
# round-6 call 23: NT GEMM output-store cache policy: plain (shipped) vs sc1 (line dropped from L2) vs nt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b23
mkdir -p $O
timeout -k 10 400 python -u tools/gemm_ab.py --only QK,Y,G,dX --rounds 9 --libs base=sir-gcn_amd/lib/libsirconv.so sc1=sir-gcn_amd/lib/libsirconv_sc1.so nt=sir-gcn_amd/lib/libsirconv_ntp.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt

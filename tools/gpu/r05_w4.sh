#!/bin/bash
# round-5: k_gemm_nt_w (weights loaded as deep as the data) vs k_gemm_nt_p + ablations (SIR_NT_W_ABL bits:
# 1 no data loads, 2 no weight loads, 4 no MFMAs, 8 no barriers, 16 no C stores, 32 no split arithmetic, 64 no split-wave LDS writes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_w4
mkdir -p $O
L=sir-gcn_amd/lib/libsirconv.so
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 5 --only QK,Y,G,dX --libs p=$L w=$L@SIR_GEMM_NT_ROUTE=w > $O/ab0.txt 2>&1 || { cat $O/ab0.txt; exit 1; }
grep -v amdgpu.ids $O/ab0.txt
for b in 3 4 7 19 23 55 87 31; do
  SIR_NT_W_ABL=$b timeout -k 10 200 python -u tools/gemm_ab.py --rounds 3 --only Y --libs w$b=$L@SIR_GEMM_NT_ROUTE=w > $O/ab$b.txt 2>&1 || { cat $O/ab$b.txt; exit 1; }
  grep -v "^total\|amdgpu.ids" $O/ab$b.txt
done

#!/bin/bash
# round-5: timing-only ablations of k_gemm_nt_w (SIR_NT_W_ABL bits: 1 no data loads, 2 no weight loads,
# 4 no MFMAs, 8 no barriers, 16 no C stores) on the S2 Y / QK shapes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_w2
mkdir -p $O
L=sir-gcn_amd/lib/libsirconv.so
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 3 --only QK,Y --libs p=$L w=$L@SIR_GEMM_NT_ROUTE=w > $O/ab0.txt 2>&1 || { cat $O/ab0.txt; exit 1; }
cat $O/ab0.txt
for b in 1 2 3 4 8 16 19 7 23 31; do
  SIR_NT_W_ABL=$b timeout -k 10 200 python -u tools/gemm_ab.py --rounds 3 --only QK,Y --libs w$b=$L@SIR_GEMM_NT_ROUTE=w > $O/ab$b.txt 2>&1 || { cat $O/ab$b.txt; exit 1; }
  grep -v "^total" $O/ab$b.txt
done

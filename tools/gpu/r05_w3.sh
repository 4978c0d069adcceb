#!/bin/bash
# round-5: k_gemm_nt_w (leaner split waves) vs k_gemm_nt_p on the S2 shapes + ablations (SIR_NT_W_ABL)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_w3
mkdir -p $O
L=sir-gcn_amd/lib/libsirconv.so
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 5 --only QK,Y,G,dX --libs p=$L w=$L@SIR_GEMM_NT_ROUTE=w > $O/ab0.txt 2>&1 || { cat $O/ab0.txt; exit 1; }
grep -v amdgpu.ids $O/ab0.txt
for b in 3 4 7 19 23; do
  SIR_NT_W_ABL=$b timeout -k 10 200 python -u tools/gemm_ab.py --rounds 3 --only QK,Y --libs w$b=$L@SIR_GEMM_NT_ROUTE=w > $O/ab$b.txt 2>&1 || { cat $O/ab$b.txt; exit 1; }
  grep -v "^total\|amdgpu.ids" $O/ab$b.txt
done

#!/bin/bash
# round-5: k_gemm_nt_w, each role alone (SIR_NT_W_ABL 8|256: split waves only, 8|512: MFMA waves only; 1/2 no loads, 4 no MFMAs, 16 no stores)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_w5
mkdir -p $O
L=sir-gcn_amd/lib/libsirconv.so
for b in 0 267 264 283 280 536 552 556 540; do
  SIR_NT_W_ABL=$b timeout -k 10 200 python -u tools/gemm_ab.py --rounds 3 --only Y --libs w$b=$L@SIR_GEMM_NT_ROUTE=w > $O/ab$b.txt 2>&1 || { cat $O/ab$b.txt; exit 1; }
  grep -v "^total\|amdgpu.ids" $O/ab$b.txt
done

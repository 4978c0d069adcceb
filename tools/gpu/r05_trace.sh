#!/bin/bash
set -o pipefail
O=gpurun_out/r05_trace; mkdir -p $O
for c in 2 3; do for shape in "1582 300 300 0" "1582 300 600 0" "1582 600 300 1"; do
  SIR_LT_NT=$c timeout -k 10 60 ./tools/dbg/lt_trace $shape > $O/t_${c}_${shape// /_}.txt 2>&1 || exit $?
  echo "== lt=$c $shape"; cat $O/t_${c}_${shape// /_}.txt
done; done
LT_CFGS=0,2,3 timeout -k 10 300 python -u tools/dbg/small_gemm_probe.py > $O/probe.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/probe.txt

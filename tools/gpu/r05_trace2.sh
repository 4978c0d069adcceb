#!/bin/bash
set -o pipefail
O=gpurun_out/r05_trace2; mkdir -p $O
for c in 1 2 3; do for shape in "1582 300 300 0" "791 300 300 0" "1582 300 600 0"; do
  SIR_LT_NT=$c timeout -k 10 60 ./tools/dbg/lt_trace $shape > $O/t_${c}_${shape// /_}.txt 2>&1 || exit $?
  echo "== lt=$c $shape"; grep -v "step [2-7]" $O/t_${c}_${shape// /_}.txt
done; done

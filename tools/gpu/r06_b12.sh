#!/bin/bash
# round-6 call 12: dW_R (k_max_dw_qk2) row ranges x 1 / 2 / 4 (balance vs partial count), S1 max shape
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b12
mkdir -p $O
timeout -k 10 300 python -u tools/maxdw_ab.py --forms 2,2/2,2/4 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt

#!/bin/bash
# round-6 call 24: routed dz passes with U = 2 / 4 (shipped) / 6 edge pairs in flight per wave
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b24
mkdir -p $O
timeout -k 10 400 python -u tools/maxbwd_ab.py --libs u4=sir-gcn_amd/lib/libsirconv.so u6=sir-gcn_amd/lib/libsirconv_u6.so u2=sir-gcn_amd/lib/libsirconv_u2.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt

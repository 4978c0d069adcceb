#!/bin/bash
# round-6 call 10: the stream max forward with the swizzled LDS image (SIR_MLP_SWZ=1) vs the unswizzled
# build (swz0): A/B in f32 and bf16, bit-identity, and the LDS bank-conflict counters of both
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b10
mkdir -p $O
L0=sir-gcn_amd/lib/libsirconv_swz0.so
L1=sir-gcn_amd/lib/libsirconv.so
for d in f32 bf16; do
  timeout -k 10 300 python -u tools/mlpfwd_ab.py --dtype $d --libs swz0=$L0 swz1=$L1 > $O/ab_$d.txt 2>&1 || { tail -20 $O/ab_$d.txt; exit 1; }
  cat $O/ab_$d.txt | grep -v amdgpu.ids
done
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for v in swz0 swz1; do
  L=$L0; [ $v = swz1 ] && L=$L1
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/${v}_p1 -o run --output-format csv -- python3 tools/mlpfwd_ab.py --rounds 2 --libs $v=$L > $O/${v}_p1.log 2>&1 || { tail -5 $O/${v}_p1.log; exit 1; }
done
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1; grep -A12 "mlp_fwd16r" $O/summary.txt

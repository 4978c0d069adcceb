#!/bin/bash
# round-6: where the TN GEMM (k_gemm_tn, dW_R / dW at S2) spends its time: A/B against the load-ablated
# build (SIR_ABL_TN=1: zero-record descriptors, no memory traffic) and SQ counters on the dWR shape
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06tn
mkdir -p $O
L=sir-gcn_amd/lib/libsirconv.so
timeout -k 10 200 python -u tools/gemm_ab.py --only dW --libs base=$L abl=sir-gcn_amd/lib/libsirconv_tnabl.so > $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
cat $O/ab.txt
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA SQ_WAVES"
C3="SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA"
for sh in dWR; do
  i=1
  for C in "$C1" "$C2" "$C3"; do
    timeout -s KILL 90 rocprofv3 --pmc $C -d $O/${sh}_p$i -o run --output-format csv -- python3 tools/gemm_one.py --lib $L --shape $sh --reps 3 > $O/${sh}_p$i.log 2>&1 || exit $?
    i=$((i+1))
  done
done
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt

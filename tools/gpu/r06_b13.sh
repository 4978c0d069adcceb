#!/bin/bash
# round-6 call 13: SQ counters of the hybrid max backward's kernels (route, dz passes on the queue, dW_R)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b13
mkdir -p $O
L=sir-gcn_amd/lib/libsirconv.so
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_WAVES"
C3="SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
i=1
for C in "$C1" "$C2" "$C3"; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/S1_p$i -o run --output-format csv -- python3 tools/maxbwd_ab.py --rounds 2 --libs main=$L > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1
for k in k_maxb_dz k_max_dw_qk2 k_maxb_route; do grep -A30 "== S1  $k" $O/summary.txt | grep -E "==|share|INSTS_VALU|INSTS_SALU|INSTS_LDS |LDS_IDX|BANK|WAVE_CYCLES|BUSY_CYCLES|VMEM_RD|TCC_READ"; done

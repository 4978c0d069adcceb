#!/bin/bash
# round-6 call 2: GEMM tests on the shipped NT split, SQ counters of k_max_dw_qk2 (S1 max shape)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_cfg4_gpu.py -m gpu -q -x --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_WAVES"
C3="SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
i=1
for C in "$C1" "$C2" "$C3"; do
  timeout -s KILL 150 rocprofv3 --pmc $C -d $O/dw_p$i -o run --output-format csv -- python3 tools/maxdw_ab.py --forms 2 --rounds 2 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py $O --match max_dw > $O/summary.txt 2>&1; cat $O/summary.txt

# where the persistent NT GEMM spends its cycles: SQ counters on the QK and Y shapes (one rocprofv3
# pass per counter group), plus the torch streaming floors of the same byte counts
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmcg
mkdir -p $O
L=sir-gcn_amd/lib/libsirconv.so
timeout -k 10 200 python -u tools/stream_floor.py > $O/floor.txt 2>&1 || exit $?
cat $O/floor.txt
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA SQ_WAVES"
C3="SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA"
for sh in QK Y; do
  i=1
  for C in "$C1" "$C2" "$C3"; do
    timeout -s KILL 90 rocprofv3 --pmc $C -d $O/${sh}_p$i -o run --output-format csv -- python3 tools/gemm_one.py --lib $L --shape $sh --reps 3 > $O/${sh}_p$i.log 2>&1 || exit $?
    i=$((i+1))
  done
done
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt

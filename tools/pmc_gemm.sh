set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcnt
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 90 rocprofv3 --pmc $C1 -d gpurun_out/pmcnt/p1 -o run --output-format csv -- python3 tools/gemm_ab.py --libs new=sir-gcn_amd/lib/libsirconv.so --only Y --rounds 2 > gpurun_out/pmcnt/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc $C2 -d gpurun_out/pmcnt/p2 -o run --output-format csv -- python3 tools/gemm_ab.py --libs new=sir-gcn_amd/lib/libsirconv.so --only Y --rounds 2 > gpurun_out/pmcnt/p2.log 2>&1

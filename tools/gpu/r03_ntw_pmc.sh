set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ntw_pmc
mkdir -p $O
L=sir-gcn_amd/lib
for v in new:libsirconv.so noA:libsirconv_a1.so old:libsirconv_old.so; do n=${v%%:*}; lib=$L/${v#*:}
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o run -- python3 tools/gemm_one.py --lib $lib --shape Y > $O/kt_$n.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -d $O/p1_$n -o run -- python3 tools/gemm_one.py --lib $lib --shape Y > $O/p1_$n.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/p2_$n -o run -- python3 tools/gemm_one.py --lib $lib --shape Y > $O/p2_$n.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/p3_$n -o run -- python3 tools/gemm_one.py --lib $lib --shape Y > $O/p3_$n.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum -d $O/p4_$n -o run -- python3 tools/gemm_one.py --lib $lib --shape Y > $O/p4_$n.log 2>&1 || exit 1
done
find $O -name "*.csv" | head -50

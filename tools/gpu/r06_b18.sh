#!/bin/bash
# round-6 call 18: routing-table kernel with up to 4096 blocks (16 a CU) vs 1024 (4 a CU: one wave a SIMD)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b18
mkdir -p $O
timeout -k 10 300 python -u tools/maxbwd_ab.py --libs cap4096=sir-gcn_amd/lib/libsirconv.so cap1024=sir-gcn_amd/lib/libsirconv_r1024.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/maxbwd_ab.py --rounds 2 --libs cap4096=sir-gcn_amd/lib/libsirconv.so cap1024=sir-gcn_amd/lib/libsirconv_r1024.so > $O/prof.log 2>&1 || exit $?
grep -h "maxb_route" $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | python3 -c "
import sys, csv
rows = [r for r in csv.reader(sys.stdin)]
for r in rows: pass
print(len(rows), 'route dispatches')
" || true
python3 tools/kernel_summary.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) --top 8

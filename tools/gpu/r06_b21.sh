#!/bin/bash
# round-6 call 21: the split-row combine with 16 partial rows in flight per thread (pf16) vs 4 (shipped)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b21
mkdir -p $O
for v in base pf16; do
  L=sir-gcn_amd/lib/libsirconv.so; [ $v = pf16 ] && L=sir-gcn_amd/lib/libsirconv_pf16.so
  SIRGCN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/prof_$v.log 2>&1 || exit $?
  echo "== $v"; python3 tools/kernel_summary.py $(ls $O/prof_$v/*/run_kernel_stats.csv $O/prof_$v/run_kernel_stats.csv 2>/dev/null | head -1) --top 12 | grep -E "combine|edge"
done
for rep in 1 2; do
  for v in base pf16; do
    L=sir-gcn_amd/lib/libsirconv.so; [ $v = pf16 ] && L=sir-gcn_amd/lib/libsirconv_pf16.so
    SIRGCN_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { tail -5 $O/b_${v}_$rep.err; exit 1; }
  done
  python3 -c "import json; a=json.load(open('$O/b_base_$rep.json')); b=json.load(open('$O/b_pf16_$rep.json')); print('S2 base', a['ms_per_step'], '| pf16', b['ms_per_step'])"
done

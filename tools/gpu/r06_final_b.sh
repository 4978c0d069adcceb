#!/bin/bash
# round-6 final set B: the other bench lines (S1, S2 mean / sym, S1 / S2 max in f32 and bf16, configs 1/2/3/5)
# and the cfg5 / cfg2 / S1-max (f32, bf16) kernel summaries
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/final6}
mkdir -p $O
line() { n=$1; shift; timeout -k 10 500 python -u bench.py "$@" --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'), d['value'])"; }
line S1 --graph S1 --steps 20 --warmup 5
line S2mean --agg mean --steps 20 --warmup 5
line S2sym --agg sym --steps 20 --warmup 5
line S1max --graph S1 --agg max --steps 10 --warmup 3
line S1maxbf16 --graph S1 --agg max --dtype bf16 --steps 10 --warmup 3
line S2max --graph S2 --agg max --steps 5 --warmup 2
line S2maxbf16 --graph S2 --agg max --dtype bf16 --steps 5 --warmup 2
for w in cfg1 cfg2 cfg3 cfg5; do line $w --workload $w --steps 50 --warmup 10; done
for w in cfg5 cfg2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-aux --no-capture > $O/prof_$w.log 2>&1 || exit $?
  python3 tools/kernel_summary.py $(ls $O/prof_$w/*/run_kernel_stats.csv $O/prof_$w/run_kernel_stats.csv 2>/dev/null | head -1) --top 20 > $O/${w}_summary.txt
done
for d in f32 bf16; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_S1max_$d -o run --output-format csv -- python3 bench.py --graph S1 --agg max --dtype $d --steps 3 --warmup 1 --no-cpu-baseline --no-aux > $O/prof_S1max_$d.log 2>&1 || exit $?
  python3 tools/kernel_summary.py $(ls $O/prof_S1max_$d/*/run_kernel_stats.csv $O/prof_S1max_$d/run_kernel_stats.csv 2>/dev/null | head -1) --top 20 > $O/S1max_${d}_summary.txt
done
head -12 $O/S1max_f32_summary.txt; head -12 $O/S1max_bf16_summary.txt

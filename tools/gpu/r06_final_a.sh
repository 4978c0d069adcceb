#!/bin/bash
# round-6 final set A: smoke, the default bench line (S2) + its rocprof kernel summary, the PMC
# FETCH_SIZE / WRITE_SIZE passes of the S2 f32 and bf16 steps (tools/pmc_traffic.py), the S2 bf16 line
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/final6}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
for d in f32 bf16; do
  x=""; [ $d = bf16 ] && x="--dtype bf16"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$d -o run --output-format csv -- python3 bench.py $x --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/pmc_fetch_$d.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$d -o run --output-format csv -- python3 bench.py $x --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/pmc_write_$d.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py $O/pmc_fetch_$d $O/pmc_write_$d --graph S2 --agg sum --H 256 --dtype $d --out $O/pmc_traffic_S2_$d.json > /dev/null || exit $?
done
# the bench lines read the counter files from profiles/: the fresh ones first
cp $O/pmc_traffic_S2_f32.json profiles/pmc_traffic_S2.json && cp $O/pmc_traffic_S2_bf16.json profiles/pmc_traffic_S2_bf16.json || exit 1
timeout -k 10 400 python -u bench.py > $O/b_S2.json 2> $O/b_S2.err || exit $?
python3 -c "import json; d=json.load(open('$O/b_S2.json')); print('S2', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['frac'], d['projections']['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/prof.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) --top 16 > $O/S2_summary.txt; cat $O/S2_summary.txt
timeout -k 10 400 python -u bench.py --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_S2bf16.json 2> $O/b_S2bf16.err || exit $?
python3 -c "import json; d=json.load(open('$O/b_S2bf16.json')); print('S2bf16', d['ms_per_step'], d.get('ms_per_step_median'), d.get('roofline', {}).get('frac'))"

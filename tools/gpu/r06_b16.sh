#!/bin/bash
# round-6 call 16: the gradient-link test; S1 / S2 max lines on the work-queue build (labelled hybrid);
# the S2 bf16 kernel summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b16
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_stacks_gpu.py -k grad_link -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() { n=$1; shift; timeout -k 10 500 python -u bench.py "$@" --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'), d['value'], d['config'].get('max_bwd'))"; }
line S1max --graph S1 --agg max --steps 10 --warmup 3
line S1maxbf16 --graph S1 --agg max --dtype bf16 --steps 10 --warmup 3
line S2max --graph S2 --agg max --steps 5 --warmup 2
line S2maxbf16 --graph S2 --agg max --dtype bf16 --steps 5 --warmup 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bf16 -o run --output-format csv -- python3 bench.py --dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/prof_bf16.log 2>&1 || exit $?
python3 tools/kernel_summary.py $(ls $O/prof_bf16/*/run_kernel_stats.csv $O/prof_bf16/run_kernel_stats.csv 2>/dev/null | head -1) --top 16 > $O/S2bf16_summary.txt; cat $O/S2bf16_summary.txt

#!/bin/bash
# round-6 final set C (last build): smoke, the GPU suite, the S2 headline, the max lines and the stack configs
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/final6d}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { grep -E "passed|failed|Error" $O/suite.log | tail -5; exit 1; }
grep -E "passed|failed" $O/suite.log | tail -1
line() { n=$1; shift; timeout -k 10 500 python -u bench.py "$@" --no-aux > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'), d['value'], (d.get('roofline') or {}).get('frac'))"; }
line S2
line S1max --graph S1 --agg max --steps 10 --warmup 3 --no-cpu-baseline
line S1maxbf16 --graph S1 --agg max --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline
line S2max --graph S2 --agg max --steps 5 --warmup 2 --no-cpu-baseline
line S2maxbf16 --graph S2 --agg max --dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline
for w in cfg1 cfg2 cfg3 cfg5; do line $w --workload $w --steps 50 --warmup 10 --no-cpu-baseline; done

#!/bin/bash
# round-6 call 25: the bf16 max lines with the max forward's roofline against the dense 16-bit peak
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b25
mkdir -p $O
line() { n=$1; shift; timeout -k 10 500 python -u bench.py "$@" --no-aux --no-cpu-baseline > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); r=d['roofline']; print('$n', d['ms_per_step'], d.get('ms_per_step_median'), r['frac'], r['peak'], r['kernel'])"; }
line S1maxbf16 --graph S1 --agg max --dtype bf16 --steps 10 --warmup 3
line S2maxbf16 --graph S2 --agg max --dtype bf16 --steps 5 --warmup 2
line S1max --graph S1 --agg max --steps 10 --warmup 3

#!/bin/bash
# round-6 call 20: the residual-gradient link in the arxiv order too (cfg3): tests, then cfg3 / cfg2 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b20
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stacks_gpu.py tests/test_abi_cpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in cfg3 cfg2; do
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline --no-aux > $O/b_${w}_link_$rep.json 2> $O/b_${w}_link_$rep.err || { tail -5 $O/b_${w}_link_$rep.err; exit 1; }
  timeout -k 10 300 python -u -c "
import sys, runpy; sys.path.insert(0, 'sir-gcn_amd')
import sirgcn.stacks as s; s.SIRStack.link_residual_grads = False
sys.argv = ['bench.py', '--workload', '$w', '--steps', '50', '--warmup', '10', '--no-cpu-baseline', '--no-aux']
runpy.run_path('bench.py', run_name='__main__')" > $O/b_${w}_add_$rep.json 2> $O/b_${w}_add_$rep.err || { tail -5 $O/b_${w}_add_$rep.err; exit 1; }
  python3 -c "import json; a=json.load(open('$O/b_${w}_link_$rep.json')); b=json.load(open('$O/b_${w}_add_$rep.json')); print('$w link', a['ms_per_step'], a.get('ms_per_step_median'), '| add', b['ms_per_step'], b.get('ms_per_step_median'))"
done
done

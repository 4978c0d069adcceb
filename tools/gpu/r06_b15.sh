#!/bin/bash
# round-6 call 15: cfg2 with the zinc-order residual gradients linked (resact.GradLink, D2 of
# sir_resid_act_bwd) vs autograd's add (SIRStack.link_residual_grads = False); stack tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b15
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stacks_gpu.py tests/test_abi_cpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --workload cfg2 --steps 50 --warmup 10 --no-cpu-baseline --no-aux > $O/b_link_$rep.json 2> $O/b_link_$rep.err || { tail -5 $O/b_link_$rep.err; exit 1; }
  timeout -k 10 300 python -u -c "
import sys, runpy; sys.path.insert(0, 'sir-gcn_amd')
import sirgcn.stacks as s; s.SIRStack.link_residual_grads = False
sys.argv = ['bench.py', '--workload', 'cfg2', '--steps', '50', '--warmup', '10', '--no-cpu-baseline', '--no-aux']
runpy.run_path('bench.py', run_name='__main__')" > $O/b_add_$rep.json 2> $O/b_add_$rep.err || { tail -5 $O/b_add_$rep.err; exit 1; }
  python3 -c "import json; a=json.load(open('$O/b_link_$rep.json')); b=json.load(open('$O/b_add_$rep.json')); print('cfg2 link', a['ms_per_step'], a.get('ms_per_step_median'), '| add', b['ms_per_step'], b.get('ms_per_step_median'))"
done

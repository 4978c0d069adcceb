#!/bin/bash
# round-6 call 17: dW_R on a side stream beside the edge backward (SIRConvFunction.overlap_dwr) vs serial, S2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b17
mkdir -p $O
run() { n=$1; ov=$2; shift 2
  timeout -k 10 300 python -u -c "
import sys, runpy; sys.path.insert(0, 'sir-gcn_amd')
import sirgcn.conv as c; c.SIRConvFunction.overlap_dwr = $ov
sys.argv = ['bench.py'] + sys.argv[1:]
runpy.run_path('bench.py', run_name='__main__')" "$@" --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }; }
for rep in 1 2; do
  run ov_$rep True --steps 20 --warmup 5
  run ser_$rep False --steps 20 --warmup 5
  python3 -c "import json; a=json.load(open('$O/b_ov_$rep.json')); b=json.load(open('$O/b_ser_$rep.json')); print('S2 overlap', a['ms_per_step'], a.get('ms_per_step_median'), '| serial', b['ms_per_step'], b.get('ms_per_step_median'))"
done
run ov_S1 True --graph S1 --steps 20 --warmup 5
run ser_S1 False --graph S1 --steps 20 --warmup 5
python3 -c "import json; a=json.load(open('$O/b_ov_S1.json')); b=json.load(open('$O/b_ser_S1.json')); print('S1 overlap', a['ms_per_step'], a.get('ms_per_step_median'), '| serial', b['ms_per_step'], b.get('ms_per_step_median'))"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cfg4_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log

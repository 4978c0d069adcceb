# small-batch route, round 2: TN variants at config-5 / config-1 shapes, the stack benches with the native
# route as product default, the S2 line (unchanged route), then the whole GPU suite
set -o pipefail
O=gpurun_out/small2
mkdir -p $O
L=sir-gcn_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -2 $O/tests.log; [ $r -eq 0 ] || exit $r
for vh in "1582 300" "5120 64"; do
  set -- $vh
  echo "== V=$1 H=$2"
  timeout -k 10 300 python -u tools/gemm_ab.py --V $1 --H $2 --rounds 5 --reps 20 --torch --only dWR,dW --libs base=$L/libsirconv.so nb1=$L/libsirconv_nb1.so w512=$L/libsirconv_w512.so nb1w2k=$L/libsirconv_nb1w2k.so || exit $?
done > $O/ab.txt 2>&1; r=$?; cat $O/ab.txt; [ $r -eq 0 ] || exit $r
for w in cfg5 cfg1 cfg2 cfg3; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$w.json 2> $O/b_$w.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$w.json')); print('$w', d['ms_per_step'], d.get('ms_per_step_median'))"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_S2.json 2> $O/b_S2.err || exit $?
python3 -c "import json; d=json.load(open('$O/b_S2.json')); print('S2', d['ms_per_step'], d.get('ms_per_step_median'), d['projections']['ms_per_step'])"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1; r=$?; tail -3 $O/suite.log; exit $r

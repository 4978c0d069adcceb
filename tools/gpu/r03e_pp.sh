# ping-pong NT GEMM (opt-in SIR_NT_PP=1): bit-identity tests vs k_gemm_nt_p, stand-alone A/B on the S2 shapes,
# then the S2 step both ways
set -o pipefail
O=gpurun_out/pp
mkdir -p $O
L=sir-gcn_amd/lib/libsirconv.so
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "pingpong" > $O/tests.log 2>&1; r=$?; tail -4 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 5 --only QK,Y,G,dX --libs p=$L@SIR_NT_PP=0 pp=$L@SIR_NT_PP=1 > $O/ab.txt 2>&1; r=$?; cat $O/ab.txt; [ $r -eq 0 ] || exit $r
for pp in 0 1; do
  SIR_NT_PP=$pp timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$pp.json 2> $O/b_$pp.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$pp.json')); print('PP=$pp', d['ms_per_step'], d.get('ms_per_step_median'), d['projections']['ms_per_step'], {k: v['ms'] for k, v in d['projections']['kernels'].items()})"
done

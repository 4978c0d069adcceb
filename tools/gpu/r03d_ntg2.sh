# DMA NT GEMM v2 (32 rows x 256 features per wave, each row split once) vs k_gemm_nt_p; S2 step both ways;
# max path and cfg5 after the elementwise / GraphNorm changes
set -o pipefail
O=gpurun_out/ntg2
mkdir -p $O
L=sir-gcn_amd/lib
SIR_NT_G=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 5 --only QK,Y,G,dX --libs ntp=$L/libsirconv.so g1=$L/libsirconv.so@SIR_NT_G=1 g2=$L/libsirconv_tb2.so@SIR_NT_G=1 > $O/ab.txt 2>&1; r=$?; cat $O/ab.txt; [ $r -eq 0 ] || exit $r
for g in 0 1; do
  SIR_NT_G=$g timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/bench_g$g.json 2> $O/bench_g$g.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_g$g.json')); print('G=$g', d['ms_per_step'], d.get('ms_per_step_median'), d['projections']['ms_per_step'], {k: v['ms'] for k, v in d['projections']['kernels'].items()})"
done
timeout -k 10 400 python -u bench.py --graph S1 --agg max --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/b_S1max.json 2> $O/b_S1max.err || exit $?
python3 -c "import json; d=json.load(open('$O/b_S1max.json')); print('S1max', d['ms_per_step'], d.get('roofline', {}).get('achieved'))"
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 30 --warmup 5 --no-cpu-baseline --no-aux > $O/b_cfg5.json 2> $O/b_cfg5.err || exit $?
python3 -c "import json; d=json.load(open('$O/b_cfg5.json')); print('cfg5', d['ms_per_step'], d.get('ms_per_step_median'))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "norm or stack or cfg or max or edgemlp" > $O/suite.log 2>&1; r=$?; tail -3 $O/suite.log; exit $r

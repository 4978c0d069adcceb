# LDS-DMA NT GEMM (sirconv_gemm_g.hip): numerics, A/B against k_gemm_nt_p, streaming floors, S2 step
set -o pipefail
O=gpurun_out/ntg
mkdir -p $O
L=sir-gcn_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 5 --libs new=$L/libsirconv.so ntp=$L/libsirconv_ntp.so mix0=$L/libsirconv_mix0.so > $O/ab.txt 2>&1; r=$?; cat $O/ab.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 200 python -u tools/stream_floor.py > $O/floor.txt 2>&1; r=$?; cat $O/floor.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], d.get('ms_per_step_median'), d['projections'])"
timeout -k 10 300 python -u -m pytest tests/test_edgemlp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/mlp_tests.log 2>&1; r=$?; tail -3 $O/mlp_tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u bench.py --graph S1 --agg max --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/b_S1max.json 2> $O/b_S1max.err || exit $?
python3 -c "import json; d=json.load(open('$O/b_S1max.json')); print('S1max', d['ms_per_step'], {k: v.get('ms') for k, v in d.get('kernels', {}).items()})"
bash tools/gpu/r03d_cfg.sh || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1; r=$?; tail -4 $O/suite.log; exit $r

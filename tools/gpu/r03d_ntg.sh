# LDS-DMA NT GEMM (sirconv_gemm_g.hip): numerics, A/B against k_gemm_nt_p, streaming floors, S2 step
set -o pipefail
O=gpurun_out/ntg
mkdir -p $O
L=sir-gcn_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 5 --only QK,Y,G,dX --libs dma=$L/libsirconv.so ntp=$L/libsirconv_ntp.so > $O/ab.txt 2>&1; r=$?; cat $O/ab.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 200 python -u tools/stream_floor.py > $O/floor.txt 2>&1; r=$?; cat $O/floor.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], d.get('ms_per_step_median'), d['projections'])"

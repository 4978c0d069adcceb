# Forward sign-mask words by v_writelane (libsirconv.so) vs per-lane selects (libsirconv_sel.so),
# bf16 forward UNROLL 8 (fh8), bf16 dK pass with per-lane mask loads and 16 edges per batch (dk16):
# interleaved A/B on S2, then the sign-mask and forward parity tests and S2 bench lines.
set -o pipefail
mkdir -p gpurun_out/wl
O=gpurun_out/wl
L=sir-gcn_amd/lib
ab() { name=$1; shift; timeout -k 10 400 python -u tools/edge_ab.py --graph S2 "$@" > $O/ab_$name.txt 2>&1; r=$?; echo "$name rc=$r"; tail -4 $O/ab_$name.txt; return $r; }
ab f32_sum --agg sum --libs sel=$L/libsirconv_sel.so wl=$L/libsirconv.so || exit $?
ab bf16_sum --agg sum --dtype bf16 --libs sel=$L/libsirconv_sel.so wl=$L/libsirconv.so || exit $?
ab f32_sym --agg sym --libs sel=$L/libsirconv_sel.so wl=$L/libsirconv.so || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_amp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -2 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_S2.json 2> $O/b_S2.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_S2.json
timeout -k 10 300 python -u bench.py --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_S2bf16.json 2> $O/b_S2bf16.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_S2bf16.json

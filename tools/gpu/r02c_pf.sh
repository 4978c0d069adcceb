# Software-pipelined edge indices (forward col[], dK col[]/perm[]; libsirconv.so) vs none (libsirconv_nopf.so):
# interleaved A/B on S2 and S1, then the GPU parity suite.
set -o pipefail
mkdir -p gpurun_out/pf
O=gpurun_out/pf
L=sir-gcn_amd/lib
ab() { name=$1; shift; timeout -k 10 400 python -u tools/edge_ab.py "$@" > $O/ab_$name.txt 2>&1; r=$?; echo "$name rc=$r"; grep -v amdgpu.ids $O/ab_$name.txt | tail -3; return $r; }
ab f32_sum --graph S2 --agg sum --libs nopf=$L/libsirconv_nopf.so pf=$L/libsirconv.so || exit $?
ab bf16_sum --graph S2 --agg sum --dtype bf16 --libs nopf=$L/libsirconv_nopf.so pf=$L/libsirconv.so || exit $?
ab f32_sym --graph S2 --agg sym --libs nopf=$L/libsirconv_nopf.so pf=$L/libsirconv.so || exit $?
ab f32_mean --graph S2 --agg mean --libs nopf=$L/libsirconv_nopf.so pf=$L/libsirconv.so || exit $?
ab S1u --graph S1u --agg sum --libs nopf=$L/libsirconv_nopf.so pf=$L/libsirconv.so || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -2 $O/tests.log; exit $r

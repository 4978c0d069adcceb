# dQ pass with prefetched scalar mask loads (libsirconv.so) vs the wide vector form (vmask); S2 sum / mean / bf16 / S1; sign-mask tests
set -o pipefail
mkdir -p gpurun_out/dqs
O=gpurun_out/dqs
L=sir-gcn_amd/lib
ab() { name=$1; shift; timeout -k 10 400 python -u tools/edge_ab.py "$@" > $O/ab_$name.txt 2>&1; r=$?; echo "$name rc=$r"; grep -v amdgpu.ids $O/ab_$name.txt | tail -2; return $r; }
ab f32_sum --graph S2 --agg sum --libs vmask=$L/libsirconv_vmask.so smem=$L/libsirconv.so || exit $?
ab bf16_sum --graph S2 --agg sum --dtype bf16 --libs vmask=$L/libsirconv_vmask.so smem=$L/libsirconv.so || exit $?
ab f32_mean --graph S2 --agg mean --libs vmask=$L/libsirconv_vmask.so smem=$L/libsirconv.so || exit $?
ab S1 --graph S1 --agg sum --libs vmask=$L/libsirconv_vmask.so smem=$L/libsirconv.so || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_amp_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -2 $O/tests.log; exit $r

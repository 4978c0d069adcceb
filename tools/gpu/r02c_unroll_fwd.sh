# fp32 forward rows in flight per wave after the writelane / buffer-gather / col-prefetch changes: 6, 5, 3 vs 4
set -o pipefail
mkdir -p gpurun_out/ufwd
O=gpurun_out/ufwd
L=sir-gcn_amd/lib
timeout -k 10 600 python -u tools/edge_ab.py --graph S2 --agg sum --libs base=$L/libsirconv.so ff6=$L/libsirconv_ff6.so ff5=$L/libsirconv_ff5.so ff3=$L/libsirconv_ff3.so > $O/ab_sum.txt 2>&1; r=$?; grep -v amdgpu.ids $O/ab_sum.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u tools/edge_ab.py --graph S2 --agg sym --libs base=$L/libsirconv.so ff6=$L/libsirconv_ff6.so ff5=$L/libsirconv_ff5.so > $O/ab_sym.txt 2>&1; r=$?; grep -v amdgpu.ids $O/ab_sym.txt; exit $r

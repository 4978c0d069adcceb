# dK pass rows in flight per wave with the prefetched indices: 16-bit 6 (sh6), 5, 4 vs 8; fp32 6, 4 vs 8
set -o pipefail
mkdir -p gpurun_out/usrc
O=gpurun_out/usrc
L=sir-gcn_amd/lib
timeout -k 10 600 python -u tools/edge_ab.py --graph S2 --agg sum --dtype bf16 --libs base=$L/libsirconv.so sh6=$L/libsirconv_sh6.so sh5=$L/libsirconv_sh5.so sh4=$L/libsirconv_sh4.so > $O/ab_bf16.txt 2>&1; r=$?; grep -v amdgpu.ids $O/ab_bf16.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u tools/edge_ab.py --graph S2 --agg sum --libs base=$L/libsirconv.so ss6=$L/libsirconv_ss6.so ss4=$L/libsirconv_ss4.so > $O/ab_f32.txt 2>&1; r=$?; grep -v amdgpu.ids $O/ab_f32.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u tools/edge_ab.py --graph S2 --agg sym --libs base=$L/libsirconv.so ss6=$L/libsirconv_ss6.so > $O/ab_f32sym.txt 2>&1; r=$?; grep -v amdgpu.ids $O/ab_f32sym.txt; exit $r

# confirm the fp32 forward UNROLL 6 (ff6) vs 4 (base) with more rounds, S2 and S1
set -o pipefail
mkdir -p gpurun_out/ufwd2
O=gpurun_out/ufwd2
L=sir-gcn_amd/lib
timeout -k 10 600 python -u tools/edge_ab.py --graph S2 --agg sum --rounds 11 --libs base=$L/libsirconv.so ff6=$L/libsirconv_ff6.so > $O/ab_S2.txt 2>&1; r=$?; grep -v amdgpu.ids $O/ab_S2.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u tools/edge_ab.py --graph S1 --agg sum --rounds 11 --libs base=$L/libsirconv.so ff6=$L/libsirconv_ff6.so > $O/ab_S1.txt 2>&1; r=$?; grep -v amdgpu.ids $O/ab_S1.txt; exit $r

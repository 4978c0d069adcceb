# k_combine with 8 partial rows in flight per thread (libsirconv.so) vs 4 (cpf4); S2 sum / sym, bf16
set -o pipefail
mkdir -p gpurun_out/comb
O=gpurun_out/comb
L=sir-gcn_amd/lib
ab() { name=$1; shift; timeout -k 10 400 python -u tools/edge_ab.py "$@" > $O/ab_$name.txt 2>&1; r=$?; echo "$name rc=$r"; grep -v amdgpu.ids $O/ab_$name.txt | tail -2; return $r; }
ab f32_sum --graph S2 --agg sum --libs cpf4=$L/libsirconv_cpf4.so cpf8=$L/libsirconv.so || exit $?
ab f32_sym --graph S2 --agg sym --libs cpf4=$L/libsirconv_cpf4.so cpf8=$L/libsirconv.so || exit $?
ab bf16_sum --graph S2 --agg sum --dtype bf16 --libs cpf4=$L/libsirconv_cpf4.so cpf8=$L/libsirconv.so || exit $?

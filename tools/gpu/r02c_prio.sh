# one-launch backward: wave priority for the dK waves (prio1) or the dQ waves (prio2) vs none
set -o pipefail
mkdir -p gpurun_out/prio
O=gpurun_out/prio
L=sir-gcn_amd/lib
ab() { name=$1; shift; timeout -k 10 400 python -u tools/edge_ab.py "$@" > $O/ab_$name.txt 2>&1; r=$?; echo "$name rc=$r"; grep -v amdgpu.ids $O/ab_$name.txt | tail -3; return $r; }
ab f32_sum --graph S2 --agg sum --libs base=$L/libsirconv.so prio1=$L/libsirconv_prio1.so prio2=$L/libsirconv_prio2.so || exit $?
ab bf16_sum --graph S2 --agg sum --dtype bf16 --libs base=$L/libsirconv.so prio1=$L/libsirconv_prio1.so prio2=$L/libsirconv_prio2.so || exit $?
ab f32_sym --graph S2 --agg sym --libs base=$L/libsirconv.so prio1=$L/libsirconv_prio1.so prio2=$L/libsirconv_prio2.so || exit $?

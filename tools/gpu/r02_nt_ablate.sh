# Persistent NT GEMM: setprio variants and timing-only ablations (3: no A loads / C stores,
# 4: no split arithmetic, 8: no MFMAs), interleaved in one process at the S2 shapes.
set -o pipefail
mkdir -p gpurun_out
L=sir-gcn_amd/lib
timeout -k 10 400 python -u tools/gemm_ab.py --rounds 5 --libs base=$L/libsirconv.so prio1=$L/libsirconv_prio1.so prio2=$L/libsirconv_prio2.so noldst=$L/libsirconv_abl3.so nosplit=$L/libsirconv_abl4.so nomfma=$L/libsirconv_abl8.so > gpurun_out/ab_nt_ablate.txt 2>&1; r=$?; grep -v amdgpu.ids gpurun_out/ab_nt_ablate.txt; exit $r

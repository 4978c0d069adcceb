# Persistent NT GEMM (SIR_NT_PERSIST=1, libsirconv.so) vs the per-tile launch (libsirconv_ntclassic.so):
# interleaved A/B at the S2 shapes, the GEMM numerics tests, then one S2 bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_ab.py --libs classic=sir-gcn_amd/lib/libsirconv_ntclassic.so persist=sir-gcn_amd/lib/libsirconv.so > gpurun_out/ab_nt_persist.txt 2>&1; r=$?; cat gpurun_out/ab_nt_persist.txt | grep -v amdgpu.ids; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gemm.txt 2>&1; r=$?; tail -3 gpurun_out/t_gemm.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_S2_persist.json 2> gpurun_out/b_S2_persist.err; r=$?; tail -c 1500 gpurun_out/b_S2_persist.json; exit $r

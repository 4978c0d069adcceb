# small-batch GEMM route (k_gemm_nt_s / k_gemm_tn_s): GEMM tests, then timings of the small route vs the
# block-tiled kernels vs torch (hipBLASLt) at config-5 (V 1582, H 300), config-1 (V 5120, H 64), and
# 16k / 33k-row shapes (the threshold), then the cfg5 / cfg1 bench lines with the native route
set -o pipefail
O=gpurun_out/small
mkdir -p $O
L=sir-gcn_amd/lib/libsirconv.so
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -5 $O/tests.log; [ $r -eq 0 ] || exit $r
for vh in "1582 300" "5120 64" "5120 128" "16384 256" "33000 256"; do
  set -- $vh
  echo "== V=$1 H=$2"
  timeout -k 10 300 python -u tools/gemm_ab.py --V $1 --H $2 --rounds 5 --reps 20 --torch --libs small=$L@SIR_GEMM_SMALL_ROWS=1000000000 block=$L@SIR_GEMM_SMALL_ROWS=0 || exit $?
done > $O/ab.txt 2>&1; r=$?; cat $O/ab.txt; exit $r

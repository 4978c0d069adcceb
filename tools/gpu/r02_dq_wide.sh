# dQ pass, wide mask chunks (SIR_DQ_WIDE=1, libsirconv.so) vs the per-batch form (libsirconv_narrow.so):
# interleaved A/B on S2 (sum, sym, bf16 sum), then the sign-mask bit-identity tests.
set -o pipefail
mkdir -p gpurun_out
ab() { name=$1; shift; timeout -k 10 400 python -u tools/edge_ab.py --graph S2 --libs narrow=sir-gcn_amd/lib/libsirconv_narrow.so wide=sir-gcn_amd/lib/libsirconv.so "$@" > gpurun_out/ab_$name.txt 2>&1; r=$?; echo "$name rc=$r"; cat gpurun_out/ab_$name.txt | tail -3; return $r; }
ab dq_sum --agg sum || exit $?
ab dq_sym --agg sym || exit $?
ab dq_bf16 --agg sum --dtype bf16 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "sign_mask or one_launch" > gpurun_out/t_mask.txt 2>&1; r=$?; tail -3 gpurun_out/t_mask.txt; exit $r

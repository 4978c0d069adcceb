# weight-resident persistent split-fp16 edge-MLP forward vs the per-item one (A/B libraries)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mlp2
mkdir -p $O
L=sir-gcn_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_edgemlp_gpu.py tests/test_stacks_gpu.py -x -q --timeout 200 --timeout-method thread -k "edgemlp or max or seq or dictionary or cfg1 or fused" > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
for lib in libsirconv libsirconv_nores; do
  SIRGCN_LIB=$L/$lib.so timeout -k 10 400 python -u bench.py --graph S1 --agg max --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/b_$lib.json 2> $O/b_$lib.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$lib.json')); r=d['roofline']; print('$lib', d['ms_per_step'], r['achieved'], r['frac'], r['ms_per_launch'])"
  SIRGCN_LIB=$L/$lib.so timeout -k 10 300 python -u bench.py --workload cfg1 --steps 30 --warmup 5 --no-cpu-baseline --no-aux > $O/c1_$lib.json 2> $O/c1_$lib.err || exit $?
  python3 -c "import json; d=json.load(open('$O/c1_$lib.json')); print('cfg1 $lib', d['ms_per_step'], d.get('ms_per_step_median'))"
done
# timing-only ablation: k_gemm_nt_p without its C stores (outputs meaningless) — is the store burst the wall?
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 5 --only QK,Y,dX --libs base=$L/libsirconv.so nostore=$L/libsirconv_nost.so > $O/ab_nostore.txt 2>&1; r=$?; cat $O/ab_nostore.txt; exit $r

# max path: split-fp16 forward vs the fp32-MFMA forward (A/B libraries), the backward routes, rocprof
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/max
mkdir -p $O
L=sir-gcn_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_edgemlp_gpu.py tests/test_amp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
for lib in libsirconv libsirconv_mlp32; do
  SIRGCN_LIB=$L/$lib.so timeout -k 10 400 python -u bench.py --graph S1 --agg max --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/b_$lib.json 2> $O/b_$lib.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$lib.json')); print('$lib', d['ms_per_step'], d.get('roofline', {}).get('achieved'), {k: (v.get('ms'), v.get('launches')) for k, v in d.get('kernels', {}).items()})"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --graph S1 --agg max --steps 3 --warmup 1 --no-cpu-baseline --no-aux > $O/prof.log 2>&1 || exit $?
python3 tools/kernel_summary.py $O/prof/run_kernel_stats.csv --top 25
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1; r=$?; tail -4 $O/suite.log; exit $r

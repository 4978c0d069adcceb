# one-launch MEAN backward (on G / deg): parity tests, then the S2 mean bench line
set -o pipefail
mkdir -p gpurun_out/mean
O=gpurun_out/mean
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_amp_gpu.py tests/test_stacks_gpu.py tests/test_dgl_surface_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -2 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u bench.py --agg mean --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_S2mean.json 2> $O/b_S2mean.err || exit $?
grep -o '"ms_per_step": [0-9.]*' $O/b_S2mean.json | head -1

# autocast whole-layer function: AMP / stack tests, then cfg2 and the S2 bf16 line
timeout -k 10 600 python -u -m pytest tests/test_amp_gpu.py tests/test_stacks_gpu.py tests/test_gpu_parity.py -m gpu --maxfail=20 -v --timeout 300 --timeout-method thread > gpurun_out/t10.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t10.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --workload cfg2 --steps 20 --warmup 5 > gpurun_out/b10_cfg2.json 2> gpurun_out/b10_cfg2.err || exit $?
timeout -k 10 400 python -u bench.py --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-aux > gpurun_out/b10_S2bf16.json 2> gpurun_out/b10_S2bf16.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t10b.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --graph S1 --agg max --steps 10 --warmup 3 --no-aux --no-cpu-baseline > gpurun_out/b10_S1max.json 2> gpurun_out/b10_S1max.err || exit $?

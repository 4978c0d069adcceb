# GPU suite, then the one-launch backward A/B on S2 (bench.py with and without --no-dual)
timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=25 -v --timeout 300 --timeout-method thread > gpurun_out/t5.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t5.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > gpurun_out/b5_dual.json 2> gpurun_out/b5_dual.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux --no-dual > gpurun_out/b5_nodual.json 2> gpurun_out/b5_nodual.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux --agg sym > gpurun_out/b5_dual_sym.json 2> gpurun_out/b5_dual_sym.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux --agg sym --no-dual > gpurun_out/b5_nodual_sym.json 2> gpurun_out/b5_nodual_sym.err || exit $?

# GPU suite (incl. the fused edge-MLP tests), then the S1 max-path bench line
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=30 -v --timeout 300 --timeout-method thread > gpurun_out/t7.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t7.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --graph S1 --agg max --steps 10 --warmup 3 --no-aux > gpurun_out/b7_S1max.json 2> gpurun_out/b7_S1max.err || exit $?

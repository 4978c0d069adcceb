# kernel-level profile of the cfg2 (ZINC-shaped, bf16) stack step, eager launches
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg2 -o run --output-format csv -- python3 bench.py --workload cfg2 --steps 10 --warmup 3 --no-capture > gpurun_out/prof_cfg2.json 2> gpurun_out/prof_cfg2.err || exit $?
timeout -k 10 300 python -u bench.py --graph S1 --agg max --steps 10 --warmup 3 --no-aux --no-cpu-baseline > gpurun_out/b9_S1max.json 2> gpurun_out/b9_S1max.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_gpu.py tests/test_stacks_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t9.log 2>&1 || exit $?

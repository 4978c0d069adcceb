#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_edgemlp_gpu.py tests/test_gemm_gpu.py 2>&1 | tail -2 &&
timeout -k 10 300 python -u bench.py --graph S1 --agg max --steps 10 --warmup 3 --no-cpu-baseline --no-aux > gpurun_out/b_S1max_gate.json 2> gpurun_out/b_S1max_gate.err &&
python3 -c "import json; d=json.load(open('gpurun_out/b_S1max_gate.json')); print('S1max', d['ms_per_step'], d['roofline']['all_kernels'])"

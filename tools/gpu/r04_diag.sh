#!/bin/bash
# round 4: max-form arg-flip root cause + GPU suite with every projection on the native GEMMs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/max_argflip.py 512 512 64 leaky > gpurun_out/r04_argflip.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/max_argflip.py 256 40 4 relu >> gpurun_out/r04_argflip.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/max_argflip.py 300 24 64 gelu >> gpurun_out/r04_argflip.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_suite.log 2>&1
echo "suite rc $?"
tail -30 gpurun_out/r04_suite.log

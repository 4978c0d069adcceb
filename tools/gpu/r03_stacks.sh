set -o pipefail
O=gpurun_out/stacks
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stacks_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -4 $O/tests.log; [ $r -eq 0 ] || exit $r
bash tools/gpu/r03_ab_ntw_step.sh

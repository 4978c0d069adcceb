set -o pipefail
O=gpurun_out/mlp
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_edgemlp_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -15 $O/tests.log; exit $r

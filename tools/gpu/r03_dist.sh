set -o pipefail
O=gpurun_out/dist
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_rccl_gpu.py "tests/test_gpu_parity.py::test_edge_cut_halo_exchange_on_device" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -25 $O/tests.log; [ $r -eq 0 ] || exit $r
bash tools/gpu/r03_stacks.sh

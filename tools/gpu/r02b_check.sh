# Re-entry check: GPU suite + S2 bench from this container's fresh build.
set -o pipefail
mkdir -p gpurun_out/chk
O=gpurun_out/chk
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; r=$?; tail -3 $O/gpu_tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_S2.json 2> $O/b_S2.err || exit $?
tail -c 400 $O/b_S2.json

# full GPU suite + smoke
set -o pipefail
O=gpurun_out/suite
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -15 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; r=$?; tail -3 $O/smoke.log; exit $r

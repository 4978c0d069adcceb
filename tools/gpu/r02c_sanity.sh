# round-end rehearsal: smoke() and the whole -m gpu suite on the final build
set -o pipefail
mkdir -p gpurun_out/sanity
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/sanity/smoke.log 2>&1; r=$?; tail -2 gpurun_out/sanity/smoke.log; [ $r -eq 0 ] || exit $r
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sanity/tests.log 2>&1; r=$?; tail -2 gpurun_out/sanity/tests.log; exit $r

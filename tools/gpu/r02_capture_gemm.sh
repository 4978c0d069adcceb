# stack workloads with HIP-graph replay, and the per-shape GEMM table at S2 shapes
run() { name=$1; shift; timeout -k 10 420 python -u bench.py "$@" > gpurun_out/g_$name.json 2> gpurun_out/g_$name.err; r=$?; echo "$name rc=$r"; return $r; }
run cfg1 --workload cfg1 --steps 50 --warmup 5 || exit $?
run cfg2 --workload cfg2 --steps 20 --warmup 5 || exit $?
run cfg3 --workload cfg3 --steps 20 --warmup 5 || exit $?
run cfg5 --workload cfg5 --steps 50 --warmup 5 || exit $?
timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/gemm_shapes.txt 2>&1 || exit $?

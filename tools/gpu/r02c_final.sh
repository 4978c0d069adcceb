# Round-2 (session 3) measurement set from one build on one box: bench lines (S2 headline with cpu_baseline,
# S1, controls, BASELINE configs), rocprofv3 kernel-trace stats and PMC traffic for S2 and S1.
set -o pipefail
mkdir -p gpurun_out/final5
O=gpurun_out/final5
run() { name=$1; shift; timeout -k 10 420 python -u bench.py "$@" > $O/b_$name.json 2> $O/b_$name.err; r=$?; echo "$name rc=$r $(tail -c 300 $O/b_$name.json | tr -d '\n' | cut -c1-120)"; return $r; }
run S2 --steps 20 --warmup 5 || exit $?
run S1 --graph S1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
run S1u --graph S1u --steps 20 --warmup 5 --no-cpu-baseline --no-aux || exit $?
run S2mean --agg mean --steps 20 --warmup 5 --no-cpu-baseline --no-aux || exit $?
run S2sym --agg sym --steps 20 --warmup 5 --no-cpu-baseline --no-aux || exit $?
run S2bf16 --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-aux || exit $?
run S1max --graph S1 --agg max --steps 10 --warmup 3 --no-cpu-baseline --no-aux || exit $?
run cfg1 --workload cfg1 --steps 50 --warmup 5 || exit $?
run cfg2 --workload cfg2 --steps 20 --warmup 5 || exit $?
run cfg3 --workload cfg3 --steps 20 --warmup 5 || exit $?
run cfg5 --workload cfg5 --steps 50 --warmup 5 || exit $?
BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline" bash tools/profile_round.sh $O/S2 || exit $?
BENCH_ARGS="--graph S1 --steps 5 --warmup 2 --no-cpu-baseline" bash tools/profile_round.sh $O/S1 || exit $?
echo done

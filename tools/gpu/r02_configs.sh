# BASELINE configs as bench lines (cfg1/2/3/5 stacks), the S2 headline with the CPU reference dataflow on S1,
# and the S1 / S1u / mean / sym control lines.
set -o pipefail
run() { name=$1; shift; timeout -k 10 420 python -u bench.py "$@" > gpurun_out/c_$name.json 2> gpurun_out/c_$name.err; r=$?; echo "$name rc=$r"; return $r; }
run cfg1 --workload cfg1 --steps 20 --warmup 5 || exit $?
run cfg2 --workload cfg2 --steps 20 --warmup 5 || exit $?
run cfg3 --workload cfg3 --steps 20 --warmup 5 || exit $?
run cfg5 --workload cfg5 --steps 20 --warmup 5 || exit $?
run S2 --steps 20 --warmup 5 || exit $?
run S1 --graph S1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
run S1u --graph S1u --steps 20 --warmup 5 --no-cpu-baseline --no-aux || exit $?
run S2mean --agg mean --steps 20 --warmup 5 --no-cpu-baseline --no-aux || exit $?
run S2sym --agg sym --steps 20 --warmup 5 --no-cpu-baseline --no-aux || exit $?
run S2bf16 --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-aux || exit $?

# round-3 measurement set, part B: bf16 PMC + the other bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/finalB
mkdir -p $O
BENCH_ARGS="--dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-aux" bash tools/profile_round.sh $O/S2bf16 || exit $?
cp $O/S2bf16/pmc_traffic_S2_bf16.json profiles/ || exit $?
for a in "S2bf16:--dtype bf16" "S1:--graph S1" "S1u:--graph S1u" "S2mean:--agg mean" "S2sym:--agg sym" "S1max:--graph S1 --agg max" "cfg1:--workload cfg1" "cfg2:--workload cfg2" "cfg3:--workload cfg3" "cfg3nodrop:--workload cfg3 --dropout 0" "cfg5:--workload cfg5"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 400 python -u bench.py $x --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', d['ms_per_step'], d.get('ms_per_step_median'), d.get('roofline', {}).get('frac'))"
done

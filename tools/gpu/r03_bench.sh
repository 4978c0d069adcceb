# bench lines: S2 (headline), S2 with feat_dropout, cfg3 with / without dropout, cfg5, cfg2
set -o pipefail
O=gpurun_out/bench
mkdir -p $O
for a in "S2:" "S2drop:--dropout 0.2" "cfg3:--workload cfg3" "cfg3nodrop:--workload cfg3 --dropout 0" "cfg5:--workload cfg5" "cfg2:--workload cfg2" "S2bf16:--dtype bf16"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 300 python -u bench.py $x --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/b_$n.json 2> $O/b_$n.err || exit $?
  echo "$n $(python3 -c "import json,sys; d=json.load(open('$O/b_$n.json')); print(d['ms_per_step'], d.get('ms_per_step_median'), d.get('projections',{}).get('ms_per_step'))")"
done

# S2 step with the weight-resident NT kernel opted in (SIR_NT_W=1) and off (default), alternating in one call
set -o pipefail
O=gpurun_out/abstep
mkdir -p $O
for i in 1 2; do
  for w in 1 0; do
    SIR_NT_W=$w timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > $O/w${w}_$i.json 2> $O/w${w}_$i.err || exit $?
    python3 -c "import json; d=json.load(open('$O/w${w}_$i.json')); print('W=$w', d['ms_per_step'], {k: (v['ms'], v['launches']) for k, v in d['projections']['kernels'].items()})"
  done
done

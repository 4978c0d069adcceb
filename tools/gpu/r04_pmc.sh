#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE passes of the S2 f32 and bf16 steps on this build (tools/pmc_traffic.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc4
mkdir -p $O
for d in f32 bf16; do
  x=""; [ $d = bf16 ] && x="--dtype bf16"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$d -o run --output-format csv -- python3 bench.py $x --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/fetch_$d.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/write_$d -o run --output-format csv -- python3 bench.py $x --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/write_$d.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py $O/fetch_$d $O/write_$d --graph S2 --agg sum --H 256 --dtype $d --out $O/pmc_traffic_S2_$d.json > /dev/null || exit $?
done
python3 -c "import json; [print(d, json.load(open('$O/pmc_traffic_S2_%s.json' % d))['kernels']['sir_edge_agg_fwd']['hbm_bytes_per_launch']) for d in ('f32', 'bf16')]"

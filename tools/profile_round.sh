#!/bin/bash
# Profiling recipe used for profiles/ (run on the MI355X box from the repo root):
#   kernel trace + stats, then one PMC pass per counter (FETCH_SIZE and WRITE_SIZE cannot share
#   a pass on gfx950), then per-launch HBM bytes -> profiles/pmc_traffic.json.
set -e
OUT=${1:-gpurun_out}
ARGS=${BENCH_ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline"}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/prof.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc_write.log" 2>&1
GRAPH=$(echo "$ARGS" | sed -n 's/.*--graph \([A-Za-z0-9]*\).*/\1/p'); GRAPH=${GRAPH:-S2}
AGG=$(echo "$ARGS" | sed -n 's/.*--agg \([a-z]*\).*/\1/p'); AGG=${AGG:-sum}
DT=$(echo "$ARGS" | sed -n 's/.*--dtype \([a-z0-9]*\).*/\1/p'); DT=${DT:-f32}
SUF=$([ "$DT" = f32 ] && echo "" || echo "_$DT")
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --graph "$GRAPH" --agg "$AGG" --dtype "$DT" --out "$OUT/pmc_traffic_$GRAPH$SUF.json" > /dev/null

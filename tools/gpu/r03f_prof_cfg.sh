# rocprof kernel summaries of the cfg2 / cfg3 / cfg1 stacks (eager steps)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/profcfg
mkdir -p $O
for w in cfg2 cfg3 cfg1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$w -o run --output-format csv -- python3 bench.py --workload $w --steps 6 --warmup 2 --no-capture --no-cpu-baseline --no-aux > $O/$w.log 2>&1 || exit $?
  python3 tools/kernel_summary.py $(ls $O/$w/*/run_kernel_stats.csv $O/$w/run_kernel_stats.csv 2>/dev/null | head -1) --top 30 > $O/${w}_summary.txt; echo "== $w"; cat $O/${w}_summary.txt
done

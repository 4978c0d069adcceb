# rocprofv3 kernel-trace stats of the S2 bf16 (autocast) and fp32 steps
set -o pipefail
mkdir -p gpurun_out/pb
O=gpurun_out/pb
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bf16 -o run --output-format csv -- python3 bench.py --dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/bf16.log 2>&1 || exit $?
f=$(ls $O/bf16/*kernel_stats.csv | head -1); python3 tools/kernel_summary.py $f --top 30 > $O/bf16_summary.txt; cat $O/bf16_summary.txt

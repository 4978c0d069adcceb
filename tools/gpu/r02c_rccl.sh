# RCCL rehearsal of the edge-cut layer: 2 and 3 ranks sharing the box's one GPU (correctness only)
set -o pipefail
mkdir -p gpurun_out/rccl
timeout -k 10 240 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/rccl_probe.py > gpurun_out/rccl/w2.log 2>&1; r=$?; grep "rccl_probe\|Error\|error" gpurun_out/rccl/w2.log | head -30; [ $r -eq 0 ] || exit $r
timeout -k 10 240 python -m torch.distributed.run --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 tools/rccl_probe.py > gpurun_out/rccl/w3.log 2>&1; r=$?; grep "rccl_probe\|Error\|error" gpurun_out/rccl/w3.log | head -30; exit $r

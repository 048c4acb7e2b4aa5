#!/bin/bash
# Rehearsal of the N > 1 bench path on a one-GPU box: 2 ranks share cuda:0, exchange through gloo.
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --files-per-gpu ${FILES:-4} --backend gloo \
  > gpurun_out/n2.log 2>&1
rc=$?
tail -4 gpurun_out/n2.log
exit $rc

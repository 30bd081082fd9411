#!/bin/bash
# 2 ranks on one node (RCCL over xGMI with GPUs, gloo without)
python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc-per-node 2 \
    "$(dirname "$0")/distributed_data_parallel.py" "$@"

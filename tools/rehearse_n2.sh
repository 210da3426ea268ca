#!/bin/bash
# bench.py's multi-rank path on a 1-GPU box: 2 ranks, both on device 0, gloo.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
EDV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 1 > $O/rehearse_n2.json 2> $O/rehearse_n2.err \
  || { tail -30 $O/rehearse_n2.err; exit 1; }
cat $O/rehearse_n2.json

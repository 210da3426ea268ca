#!/bin/bash
# bench.py's multi-rank path on a 1-GPU box: 2 ranks, both on device 0, gloo
# (RCCL refuses two ranks on one GPU): C2 weak scaling and C3 (--total) strong
# scaling with the accept all-gather checked.  Outputs under gpurun_out/r02/$TAG/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r02/${TAG:-multi}; mkdir -p $O; cd $R
run() {
  EDV_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $1 bench.py --gpus 2 --steps 5 --reps 3 --warmup 1 --warmup-seconds 0 $2 \
    > $O/$3.json 2> $O/$3.err || { tail -30 $O/$3.err; exit 1; }
  tail -1 $O/$3.json
}
run 29555 "" n2_c2 && run 29556 "--total 1048576" n2_c3

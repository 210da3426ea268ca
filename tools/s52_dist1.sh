#!/bin/bash
# torch-free stream test + bench's multi-rank path (torch.cuda + RCCL beside
# libedv in one process) with one rank on a one-GPU box
set -o pipefail
O=gpurun_out/r02/s52
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_authn.py -v -m gpu --timeout 200 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python3 -c "import torch; print('torch sees', torch.cuda.device_count(), torch.cuda.is_available())" > $O/torch.log 2>&1; cat $O/torch.log
EDV_BENCH_FORCE_DIST=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 --steps 10 --warmup 2 --no-e2e --no-cpu-baseline \
  > $O/bench_dist1.json 2> $O/bench_dist1.err || { tail -30 $O/bench_dist1.err; exit 1; }
tail -c 400 $O/bench_dist1.json

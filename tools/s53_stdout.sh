#!/bin/bash
# bench.py under torch.distributed.run: stdout must be exactly one JSON line
# (RCCL's banner goes to stderr); one RCCL rank, then two gloo ranks on one GPU
set -o pipefail
O=gpurun_out/r02/s53
mkdir -p $O
EDV_BENCH_FORCE_DIST=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 1 --steps 10 --warmup 2 --no-e2e --no-cpu-baseline \
  > $O/dist1.out 2> $O/dist1.err || { tail -30 $O/dist1.err; exit 1; }
EDV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 2 --steps 5 --warmup 1 \
  > $O/gloo2.out 2> $O/gloo2.err || { tail -30 $O/gloo2.err; exit 1; }
for f in dist1 gloo2; do
  python3 -c "
import json, sys
lines = open('$O/$f.out').read().splitlines()
assert len(lines) == 1, lines[:3]
d = json.loads(lines[0]); print('$f', len(lines), 'line', d['n_gpus'], round(d['value'] / 1e6, 2), d['verdicts_as_expected'])"
done

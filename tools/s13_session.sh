#!/bin/bash
# s13: C4 sequential vs pipelined (bench leg), cProfile of the C5 overlap pool
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r03/s13; mkdir -p $O; cd $R
timeout -k 10 400 python3 bench.py --no-e2e --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['c4']; print('C2', d['value']); print('c4', c['verifies_per_s'], c['pipelined']); print('c5', d['c5']['summary'])"
timeout -k 10 300 python3 tools/prof_pool.py gpu_batched_overlap 20000 > $O/prof_pool_overlap.txt 2>&1 || { tail -20 $O/prof_pool_overlap.txt; exit 1; }
head -45 $O/prof_pool_overlap.txt
# C3 at full size on this one GPU: default chunk (2^18) and 2^20 per launch
for CH in 262144 1048576; do
  EDV_CHUNK=$CH timeout -k 10 300 python3 bench.py --total 16777216 --steps 3 --reps 3 --no-e2e --no-extra --no-cpu-baseline \
    > $O/c3_chunk$CH.json 2> $O/c3_chunk$CH.err || { tail -20 $O/c3_chunk$CH.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_chunk$CH.json')); print('C3 chunk $CH', d['value'], d['verdicts_as_expected'], d['timing']['gap_ms_per_step'], d['roofline']['prep_kernel_ms'], d['roofline']['main_kernel_ms'])"
done

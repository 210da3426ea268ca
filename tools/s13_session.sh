#!/bin/bash
# s13: C4 sequential vs pipelined (bench leg), cProfile of the C5 overlap pool
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r03/s13; mkdir -p $O; cd $R
timeout -k 10 400 python3 bench.py --no-e2e --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['c4']; print('C2', d['value']); print('c4', c['verifies_per_s'], c['pipelined']); print('c5', d['c5']['summary'])"
timeout -k 10 300 python3 tools/prof_pool.py gpu_batched_overlap 20000 > $O/prof_pool_overlap.txt 2>&1 || { tail -20 $O/prof_pool_overlap.txt; exit 1; }
head -45 $O/prof_pool_overlap.txt

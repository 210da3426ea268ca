#!/bin/bash
# s19: A/B of the software-pipelined SHA-512 schedule (EDV_SHA_PIPE) at C2 and C4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r03/s19; mkdir -p $O; cd $R
for round in 1 2; do
  for L in libedv.so variants/libedv_shapipe.so; do
    EDV_LIB=$R/indy-plenum_amd/$L timeout -k 10 150 python3 bench.py --no-e2e --no-extra --no-cpu-baseline > $O/c2.json 2> $O/err.txt \
      || { echo "FAILED c2 $L"; tail -5 $O/err.txt; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2.json')); print(json.dumps({'lib': '$L', 'round': $round, 'c2': d['value'], 'prep': d['roofline']['prep_kernel_ms'], 'main': d['roofline']['main_kernel_ms'], 'ok': d['verdicts_as_expected']}))" | tee -a $O/ab.jsonl
    EDV_LIB=$R/indy-plenum_amd/$L SIZES=65536,262144 timeout -k 10 150 python3 tools/bench_c4.py > $O/c4.jsonl 2> $O/err.txt \
      || { echo "FAILED c4 $L"; tail -5 $O/err.txt; exit 1; }
    python3 -c "
import json
for l in open('$O/c4.jsonl'):
    d=json.loads(l); print(json.dumps({'lib': '$L', 'round': $round, 'c4_n': d['n'], 'c4': d['verifies_per_s'], 'prep': d['prep_ms'], 'main': d['main_ms']}))" | tee -a $O/ab.jsonl
  done
done

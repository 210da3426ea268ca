#!/bin/bash
# Main-kernel layout A/B: each library variant (EDV_LIB) at C2 sequential, C2
# pipelined, and one 2^18-request chunk (C3's per-launch size), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r03/${TAG:-abm}; mkdir -p $O; cd $R
Q="--no-e2e --no-extra --no-cpu-baseline --reps ${REPS:-5}"
# MODES: bench.py argument sets, ';'-separated ("" = the C2 default); default
# C2, C2 --pipeline and one 2^18 chunk
IFS=';' read -ra MODES <<< "${MODES_STR:-;--pipeline;--batch 262144 --steps 6}"
[ ${#MODES[@]} -eq 0 ] && MODES=("")
for round in 1 2; do
  for V in ${VARIANTS:-libedv.so}; do
    for MODE in "${MODES[@]}"; do
      EDV_LIB=$R/indy-plenum_amd/$V timeout -k 10 150 python3 bench.py $Q $MODE > $O/tmp.json 2> $O/tmp.err \
        || { echo "FAILED $V $MODE"; tail -5 $O/tmp.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open('$O/tmp.json')); print(json.dumps({'lib': '$V', 'mode': '${MODE:-sequential}', 'round': $round, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'prep_ms': d['roofline']['prep_kernel_ms'], 'main_ms': d['roofline']['main_kernel_ms'], 'ok': d.get('verdicts_as_expected')}))" | tee -a $O/ab.jsonl
    done
  done
done

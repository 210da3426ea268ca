#!/bin/bash
# Extra rocprofv3 --pmc passes over the C2 bench (one counter group per pass,
# each pass its own run, each under its own time limit), summarised per kernel
# by tools/pmc_summary.py into $O/pmc_extra_summary.json.
#   TAG=s10 PMC_GROUPS="SQC_ICACHE_HITS SQC_ICACHE_MISSES;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
#     PMC_BENCH_ARGS="--batch 262144 --steps 3" bash tools/pmc_extra.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03/${TAG:-pmcx}/${PMC_NAME:-pmcx}
mkdir -p $O
cd $R
export TMPDIR=/tmp
B="python3 $R/bench.py --steps 6 --warmup 2 --reps 1 --no-e2e --no-extra --no-cpu-baseline $PMC_BENCH_ARGS"
i=0
IFS=';' read -ra GROUPS_ <<< "$PMC_GROUPS"
for C in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/p$i -o run --output-format csv -- $B > $O/pass$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -20 $O/pass$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O > $O/../${PMC_NAME:-pmcx}_summary.json || exit 1
echo "pmc extra done: $O"

#!/bin/bash
# PMC passes over one bench run each (counters in their own runs; no trace domains).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
B="python3 $R/bench.py --steps 6 --warmup 1 --no-cpu-baseline"
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C -d $O/p$i -o run --output-format csv -- $B > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $O/p$i.log; exit 1; }
done
echo pmc done

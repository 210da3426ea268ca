#!/bin/bash
# A/B of library variants built in-tree (EDV_LIB selects the .so): batch sweep each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for V in ${VARIANTS:-libedv.so}; do
  echo "== $V" >> $O/ab.log
  EDV_LIB=$R/indy-plenum_amd/$V timeout -k 10 240 python3 tools/sweep_batch.py >> $O/ab.log 2>&1 || { echo "variant $V failed"; tail -20 $O/ab.log; exit 1; }
done
cat $O/ab.log

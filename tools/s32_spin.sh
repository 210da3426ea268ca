#!/bin/bash
# e2e probe with and without spin-waiting host threads
set -o pipefail
O=gpurun_out/r02/s32
mkdir -p $O
timeout -k 10 200 python3 tools/e2e_probe.py > $O/e2e_yield.json 2> $O/err1 || { tail -20 $O/err1; exit 1; }
EDV_SPIN_WAIT=1 timeout -k 10 200 python3 tools/e2e_probe.py > $O/e2e_spin.json 2> $O/err2 || { tail -20 $O/err2; exit 1; }
cat $O/e2e_yield.json $O/e2e_spin.json

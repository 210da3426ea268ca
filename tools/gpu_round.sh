#!/bin/bash
# One GPU-box session for a round checkpoint: GPU parity suite (optionally the
# full >=10M-case corpus), smoke, bench, rocprofv3 kernel stats of the bench,
# and the HBM PMC passes (FETCH_SIZE, WRITE_SIZE, each in its own run).
# Every GPU step has its own time limit; the chain stops at the first failure.
#   STEPS="test smoke bench prof pmc"   (default: all)   PARITY_FULL=1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/round
mkdir -p $O
cd $R
STEPS=${STEPS:-"test smoke bench prof pmc"}
has() { [[ " $STEPS " == *" $1 "* ]]; }
log() { echo "== $1 $(date +%T)" | tee -a $O/session.log; }
if has test; then
  log pytest
  EDV_PARITY_FULL=${PARITY_FULL:-0} timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 600 \
    --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
if has smoke; then
  log smoke
  timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  cat $O/smoke.log
fi
if has bench; then
  log bench
  timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
  cat $O/bench.json
fi
export TMPDIR=/tmp
if has prof; then
  log rocprof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline > $O/prof_bench.log 2>&1 || { tail -30 $O/prof_bench.log; exit 1; }
  find $O/prof -name "*stats*"
fi
if has pmc; then
  i=0
  for C in ${PMC_SETS:-"FETCH_SIZE" "WRITE_SIZE"}; do
    i=$((i+1))
    log "pmc $C"
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $C -d $O/pmc$i -o run --output-format csv -- \
      python3 $R/bench.py --steps 6 --warmup 20 --no-cpu-baseline > $O/pmc$i.log 2>&1 || { echo "pmc $C failed"; tail -20 $O/pmc$i.log; exit 1; }
  done
fi
log done

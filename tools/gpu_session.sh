#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, batch sweep, rocprof stats.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
STEP=${STEP:-all}
run() { echo "== $1 $(date +%T)" >> $O/session.log; }
if [[ $STEP == all || $STEP == test ]]; then
  run pytest
  timeout -k 10 600 python3 -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
  run smoke
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  cat $O/smoke.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  run bench
  timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
  cat $O/bench.json
  run sweep
  timeout -k 10 300 python3 tools/sweep_batch.py > $O/sweep.log 2>&1 || { cat $O/sweep.log; exit 1; }
  cat $O/sweep.log
fi
if [[ $STEP == all || $STEP == prof ]]; then
  run rocprof
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_bench.log 2>&1 || { tail -30 $O/prof_bench.log; exit 1; }
  find $O/prof -name "*stats*" | head
fi
echo "session done"

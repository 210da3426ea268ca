#!/bin/bash
# One GPU-box session (round 2).  STEP picks the parts: test, bench, prof, pmc
# (comma list, default all).  Every GPU step has its own time limit and the
# chain stops at the first failure; outputs land in gpurun_out/r02/<tag>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-s1}
O=$R/gpurun_out/r02/$TAG
mkdir -p $O
cd $R
STEP=${STEP:-test,bench,prof,pmc}
has() { [[ ",$STEP," == *",$1,"* ]]; }
log() { echo "== $1 $(date +%T)" | tee -a $O/session.log; }
fail() { echo "FAILED: $1"; tail -40 "$2"; exit 1; }

if has test; then
  log pytest
  timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || fail pytest $O/pytest_gpu.log
  tail -3 $O/pytest_gpu.log
  log smoke
  timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
  cat $O/smoke.log
fi
if has bench; then
  log bench
  timeout -k 10 400 python3 bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
  cat $O/bench.json
fi
if has extra; then
  log extra
  timeout -k 10 600 bash -c "$EXTRA" > $O/extra.log 2>&1 || fail extra $O/extra.log
  tail -20 $O/extra.log
fi
export TMPDIR=/tmp
if has prof; then
  log rocprof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.log 2>&1 || fail rocprof $O/prof_bench.log
  find $O/prof -name "*stats*"
fi
if has pmc; then
  log pmc
  timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
  B="python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline"
  i=0
  for C in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C -d $O/pmc/p$i -o run --output-format csv -- $B > $O/pmc_p$i.log 2>&1 \
      || fail "pmc pass $i" $O/pmc_p$i.log
  done
  if grep -q "SQ_INSTS_VALU_INT32" $O/counters_list.txt; then
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MFMA_I8 \
      -d $O/pmc/p$i -o run --output-format csv -- $B > $O/pmc_p$i.log 2>&1 || echo "int32 pass failed (non-fatal)"
  fi
  python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.json || fail pmc_summary $O/pmc_summary.json
  echo pmc done
fi
echo "session done"

#!/bin/bash
# One GPU-box session (round 6).  STEP picks the parts (comma list):
#   test    pytest -m gpu + smoke()            (PYTEST_ARGS narrows it)
#   bench   the default bench.py line           (BENCH_ARGS)
#   trace   anatomy of synchronous C2 calls (kernel + copy + HIP API traces)
#   gather  PMC passes over tools/ubench_gather (counter calibration, known bytes)
#   flush   C2 launch pair with / without an Infinity-Cache flush between prep and main
#           (timing, then PMC passes per dispatch)
#   prof    rocprofv3 --kernel-trace --stats over the C2 bench (no extra legs)
#   pmc     rocprofv3 --pmc passes over the C2 bench + summary (profiles/pmc_latest.json)
#   lds     one --pmc pass of LDS / wait counters over the C2 bench (where the main kernel waits)
#   extra   $EXTRA (a command line)
# Every GPU step has its own time limit; the chain stops at the first failure.
# Outputs land in gpurun_out/r06/<TAG>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-s1}
O=$R/gpurun_out/r06/$TAG
mkdir -p $O
cd $R
STEP=${STEP:-test,bench}
has() { [[ ",$STEP," == *",$1,"* ]]; }
log() { echo "== $1 $(date +%T)" | tee -a $O/session.log; }
fail() { echo "FAILED: $1"; tail -40 "$2"; exit 1; }
QUIET="--no-e2e --no-extra --no-cpu-baseline"
export TMPDIR=/tmp

TCC1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
TCC2="FETCH_SIZE"
TCC3="WRITE_SIZE TCC_EA0_RDREQ_DRAM_sum TCC_BUBBLE_sum"
TCC4="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_WRREQ_sum"
pmc_passes() {  # name, command...
  local name=$1; shift
  local i=0
  for C in "$TCC1" "$TCC2" "$TCC3" "$TCC4"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C -d $O/$name/p$i -o run --output-format csv -- "$@" \
      > $O/$name/p$i.log 2>&1) || { echo "pmc $name pass $i failed"; tail -20 $O/$name/p$i.log; return 1; }
  done
}

if has test; then
  log pytest
  timeout -k 10 1500 python3 -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread $PYTEST_ARGS \
    > $O/pytest_gpu.log 2>&1 || fail pytest $O/pytest_gpu.log
  tail -3 $O/pytest_gpu.log
  log smoke
  timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
  cat $O/smoke.log
fi
if has trace; then
  log trace
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d $O/trace -o run \
    --output-format csv -- python3 $R/tools/trace_sync.py --calls 20 --marks $O/trace_marks.json \
    > $O/trace.log 2>&1) || fail trace $O/trace.log
  python3 tools/trace_sync.py --parse $O/trace --marks $O/trace_marks.json > $O/trace_summary.json 2>&1 \
    || fail trace_parse $O/trace_summary.json
  head -60 $O/trace_summary.json
fi
if has gather; then
  log gather
  mkdir -p $O/gather
  timeout -k 10 120 $R/tools/ubench_gather > $O/gather/plain.jsonl 2>&1 || fail gather $O/gather/plain.jsonl
  pmc_passes gather $R/tools/ubench_gather || exit 1
  cat $O/gather/plain.jsonl | head -20
fi
if has flush; then
  log flush
  mkdir -p $O/flush
  timeout -k 10 240 python3 tools/flush_probe.py --reps 5 --iters 10 > $O/flush/time.jsonl 2> $O/flush/time.err \
    || fail flush $O/flush/time.err
  tail -1 $O/flush/time.jsonl
  pmc_passes flush python3 $R/tools/flush_probe.py --reps 1 --iters 3 || exit 1
fi
if has bench; then
  log bench
  timeout -k 10 900 python3 bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
  cat $O/bench.json
fi
if has prof; then
  log prof
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
    -- python3 $R/bench.py --steps 20 $QUIET > $O/prof.log 2>&1) || fail prof $O/prof.log
  find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/rocprof_kernel_stats.csv
  head -12 $O/rocprof_kernel_stats.csv
fi
if has pmc; then
  log pmc
  i=0
  for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY" "$TCC1"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $C -d $O/pmc/p$i -o run --output-format csv \
      -- python3 $R/bench.py --steps 6 --warmup 1 $QUIET > $O/pmc_p$i.log 2>&1) \
      || { echo "pmc pass $i failed"; tail -20 $O/pmc_p$i.log; exit 1; }
  done
  python3 tools/pmc_summary.py $O/pmc $O/pmc_summary.json > /dev/null && echo "pmc summary written"
fi
if has lds; then
  log lds
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS -d $O/lds -o run --output-format csv \
    -- python3 $R/bench.py --steps 6 --warmup 1 $QUIET > $O/lds.log 2>&1) || fail lds $O/lds.log
  echo "lds pass done"
fi
if has extra; then
  log extra
  timeout -k 10 600 bash -c "$EXTRA" > $O/extra.log 2>&1 || fail extra $O/extra.log
  tail -30 $O/extra.log
fi
log done

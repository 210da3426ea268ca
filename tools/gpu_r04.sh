#!/bin/bash
# One GPU-box session (round 4).  STEP picks the parts (comma list):
#   test   pytest -m gpu + smoke()
#   bench  the default bench.py line (C2 + e2e + node path + C4 + C5 + CPU baseline)
#   spawn  N=1 through the multi-rank launcher (compare with bench: within 2 %)
#   c3     C3 at full size on this one GPU (16,777,216 requests per step)
#   prof   rocprofv3 --kernel-trace --stats over the C2 bench (no extra legs)
#   pmc    rocprofv3 --pmc passes (one counter group per pass) + summary
#   vc3    the 8-rank C3 line at full size, rehearsed on this one GPU
#          (EDV_VIRTUAL_DEVICES=8: 16,777,216 requests split 8 ways, verdicts checked)
#   extra  $EXTRA (a command line)
# Every GPU step has its own time limit; the chain stops at the first failure.
# Outputs land in gpurun_out/r04/<TAG>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-s1}
O=$R/gpurun_out/r04/$TAG
mkdir -p $O
cd $R
STEP=${STEP:-test,bench,prof}
has() { [[ ",$STEP," == *",$1,"* ]]; }
log() { echo "== $1 $(date +%T)" | tee -a $O/session.log; }
fail() { echo "FAILED: $1"; tail -40 "$2"; exit 1; }
QUIET="--no-e2e --no-extra --no-cpu-baseline"

if has test; then
  log pytest
  timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread $PYTEST_ARGS \
    > $O/pytest_gpu.log 2>&1 || fail pytest $O/pytest_gpu.log
  tail -3 $O/pytest_gpu.log
  log smoke
  timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
  cat $O/smoke.log
fi
if has bench; then
  log bench
  timeout -k 10 600 python3 bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
  cat $O/bench.json
fi
if has spawn; then
  log spawn
  timeout -k 10 300 python3 bench.py $QUIET > $O/bench_single.json 2> $O/bench_single.err || fail single $O/bench_single.err
  timeout -k 10 300 python3 bench.py --spawn --gpus 1 $QUIET > $O/bench_spawn1.json 2> $O/bench_spawn1.err \
    || fail spawn $O/bench_spawn1.err
  timeout -k 10 300 python3 bench.py $QUIET > $O/bench_single2.json 2> $O/bench_single2.err || fail single2 $O/bench_single2.err
  python3 -c "
import json,sys
a,b,c=(json.load(open('$O/'+f)) for f in ('bench_single.json','bench_spawn1.json','bench_single2.json'))
print('single %.4g  spawn %.4g  single2 %.4g  spawn/single %.4f' % (a['value'], b['value'], c['value'], 2*b['value']/(a['value']+c['value'])))"
fi
if has c3; then
  log c3
  timeout -k 10 600 python3 bench.py --total 16777216 --steps 5 --reps 3 $QUIET > $O/bench_c3_full.json \
    2> $O/bench_c3_full.err || fail c3 $O/bench_c3_full.err
  cat $O/bench_c3_full.json
fi
if has vc3; then
  log vc3
  EDV_VIRTUAL_DEVICES=8 timeout -k 10 600 python3 bench.py --gpus 8 $VC3_ARGS > $O/bench_c3_8rank_virtual.json \
    2> $O/bench_c3_8rank_virtual.err || fail vc3 $O/bench_c3_8rank_virtual.err
  cat $O/bench_c3_8rank_virtual.json
fi
if has extra; then
  log extra
  timeout -k 10 900 bash -c "$EXTRA" > $O/extra.log 2>&1 || fail extra $O/extra.log
  tail -30 $O/extra.log
fi
export TMPDIR=/tmp
if has prof; then
  log rocprof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 20 --warmup 5 $QUIET > $O/prof_bench.log 2>&1 || fail rocprof $O/prof_bench.log
  find $O/prof -name "*stats*"
fi
if has pmc; then
  log pmc
  timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
  B="python3 $R/bench.py --steps 6 --warmup 2 --reps 1 $QUIET"
  i=0
  for C in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum" $PMC_EXTRA; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C -d $O/pmc/p$i -o run --output-format csv -- $B > $O/pmc_p$i.log 2>&1 \
      || fail "pmc pass $i" $O/pmc_p$i.log
  done
  if grep -q "SQ_INSTS_VALU_INT32" $O/counters_list.txt; then
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT \
      -d $O/pmc/p$i -o run --output-format csv -- $B > $O/pmc_p$i.log 2>&1 || echo "int32 pass failed (non-fatal)"
  fi
  python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.json || fail pmc_summary $O/pmc_summary.json
  echo pmc done
fi
echo "session done"

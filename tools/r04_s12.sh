#!/bin/bash
# Round 4, session 12: HEAD (main body as a macro: ISA identical to the
# pre-refactor kernel) against the pre-refactor build, the split-path parity
# tests, then the PMC passes and the rocprof stats on HEAD's kernel sources.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04/s12; mkdir -p $O; cd $R
fail() { echo "FAILED: $1"; tail -30 "$2"; exit 1; }
for L in indy-plenum_amd/libedv.so indy-plenum_amd/variants/libedv_pre_prio.so; do
  MODES=sequential,split ROUNDS=1 EDV_LIB=$R/$L timeout -k 10 200 python3 -u tools/ab_split.py >> $O/ab.jsonl 2>> $O/ab.err \
    || fail ab $O/ab.err
done
cat $O/ab.jsonl
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "pipelined or split or golden" \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || fail pytest $O/pytest.log
tail -1 $O/pytest.log
TAG=s12 STEP=prof,pmc bash tools/gpu_r04.sh || exit 1

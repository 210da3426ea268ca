#!/bin/bash
# Round 4, session 22: kernel/copy traces showing the two overlaps kept this
# round -- the split pipeline's hash side beside the main kernel (C4), and the
# field-ordered synchronous call's point sides during the message copy.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04/s22; mkdir -p $O; cd $R
export TMPDIR=/tmp
fail() { echo "FAILED: $1"; tail -30 "$2"; exit 1; }
MODES=split ROUNDS=1 STEPS=10 REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tsplit -o run \
  --output-format csv -- python3 tools/ab_split.py > $O/tsplit.log 2>&1 || fail tsplit $O/tsplit.log
python3 tools/trace_split.py split $O/tsplit > $O/trace_split.json && cat $O/trace_split.json
ROUNDS=1 R=5 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tfields -o run \
  --output-format csv -- python3 tools/e2e_fields.py > $O/tfields.log 2>&1 || fail tfields $O/tfields.log
python3 tools/trace_split.py fields $O/tfields > $O/trace_fields.json && cat $O/trace_fields.json
echo "session done"

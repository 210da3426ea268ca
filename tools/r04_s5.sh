#!/bin/bash
# Round 4, session 5: main kernel with double-buffered LDS staging (variant
# dbuf: window w-1's per-lane entries copied during window w) against HEAD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04/s5; mkdir -p $O; cd $R
fail() { echo "FAILED: $1"; tail -30 "$2"; exit 1; }
for V in ${VARIANTS:-dbuf}; do
  EDV_LIB=$R/indy-plenum_amd/variants/libedv_$V.so EDV_PARITY_QUICK=1 timeout -k 10 300 python3 -u -m pytest \
    tests/test_gpu_parity.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/parity_$V.log 2>&1 \
    || fail parity_$V $O/parity_$V.log
  tail -1 $O/parity_$V.log
done
L="indy-plenum_amd/libedv.so"
for V in ${VARIANTS:-dbuf}; do L="$L indy-plenum_amd/variants/libedv_$V.so"; done
timeout -k 10 500 python3 -u tools/ab_bench.py $L $L > $O/ab.jsonl 2> $O/ab.err || fail ab $O/ab.err
cat $O/ab.jsonl
echo "session done"

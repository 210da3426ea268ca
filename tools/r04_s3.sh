#!/bin/bash
# Round 4, session 3: the main kernel's B entries staged through the A/R LDS
# slice (variant breuse) and with the A entry picked one doubling early
# (breuse_early), against HEAD: quick parity, then kernel times and C2 steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04/s3; mkdir -p $O; cd $R
fail() { echo "FAILED: $1"; tail -30 "$2"; exit 1; }
for V in breuse breuse_early; do
  EDV_LIB=$R/indy-plenum_amd/variants/libedv_$V.so EDV_PARITY_QUICK=1 timeout -k 10 300 python3 -u -m pytest \
    tests/test_gpu_parity.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/parity_$V.log 2>&1 \
    || fail parity_$V $O/parity_$V.log
  tail -1 $O/parity_$V.log
done
L="indy-plenum_amd/libedv.so indy-plenum_amd/variants/libedv_breuse.so indy-plenum_amd/variants/libedv_breuse_early.so"
timeout -k 10 500 python3 -u tools/ab_bench.py $L $L > $O/ab_breuse.jsonl 2> $O/ab.err || fail ab $O/ab.err
cat $O/ab_breuse.jsonl
echo "session done"

#!/bin/bash
# s18: C4 prep anatomy: the full prep kernel vs the hash side alone vs the two point sides alone
# (EDV_AB_SIDES measurement builds: their verdicts are meaningless, only prep_ms counts)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r03/s18; mkdir -p $O; cd $R
for L in libedv.so variants/libedv_hashonly.so variants/libedv_pointsonly.so; do
  EDV_SIDES_VARIANT=$([ $L = libedv.so ] || echo 1) EDV_ALLOW_MEASUREMENT_LIB=1 EDV_LIB=$R/indy-plenum_amd/$L SIZES=65536,262144 timeout -k 10 200 python3 tools/bench_c4.py > $O/c4_$(basename $L .so).jsonl 2> $O/err.txt \
    || { echo "FAILED $L"; tail -5 $O/err.txt; }
  echo "$L"; cat $O/c4_$(basename $L .so).jsonl
done

#!/bin/bash
# 4-bit windows (9-entry per-lane tables, radix-2^16 B digits): parity on the
# golden cases + one 1M corpus slice, then A/B against HEAD, alternating
set -o pipefail
O=gpurun_out/r02/s43
mkdir -p $O
V=indy-plenum_amd/variants/libedv_w4.so
EDV_LIB=$V EDV_PARITY_QUICK=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > $O/parity_w4.log 2>&1 || { tail -30 $O/parity_w4.log; exit 1; }
tail -2 $O/parity_w4.log
run() {  # tag lib
  EDV_LIB=$2 timeout -k 10 200 python3 bench.py --no-e2e --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); r=d['roofline']; print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(r['prep_kernel_ms'],4), round(r['main_kernel_ms'],4), d['verdicts_as_expected'])"
}
for k in 1 2; do
  run base$k indy-plenum_amd/libedv.so
  run w4_$k $V
done

#!/bin/bash
# early table-entry fetch in the main kernel: A/B against HEAD, alternating
set -o pipefail
O=gpurun_out/r02/s41
mkdir -p $O
V=indy-plenum_amd/variants
run() {  # tag lib
  EDV_LIB=$2 timeout -k 10 200 python3 bench.py --no-e2e --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); r=d['roofline']; print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(r['prep_kernel_ms'],4), round(r['main_kernel_ms'],4), d['verdicts_as_expected'])"
}
for k in 1 2; do
  run base$k indy-plenum_amd/libedv.so
  run ef1_$k $V/libedv_ef1.so
  run ef2_$k $V/libedv_ef2.so
done

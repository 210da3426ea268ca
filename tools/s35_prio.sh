#!/bin/bash
# pipelined submission with main-kernel issue priority and a one-wave-per-SIMD prep
set -o pipefail
O=gpurun_out/r02/s35
mkdir -p $O
V=indy-plenum_amd/variants
run() {  # tag lib args
  EDV_LIB=$2 timeout -k 10 200 python3 bench.py --no-e2e --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); r=d['roofline']; print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(r['prep_kernel_ms'],4), round(r['main_kernel_ms'],4))"
}
run base_seq indy-plenum_amd/libedv.so ""
run base_pipe indy-plenum_amd/libedv.so "--pipeline"
run prio_seq $V/libedv_prio.so ""
run prio_pipe $V/libedv_prio.so "--pipeline"
run priopad_pipe $V/libedv_priopad.so "--pipeline"
run priopad_seq $V/libedv_priopad.so ""

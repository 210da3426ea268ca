#!/bin/bash
# prep kernel time per side (EDV_AB_SIDES bit k = run side k: 0 hash, 1 A point, 2 R point)
set -o pipefail
O=gpurun_out/r02/s47
mkdir -p $O
for v in 7 1 2 6; do
  EDV_ALLOW_MEASUREMENT_LIB=1 EDV_LIB=indy-plenum_amd/variants/libedv_sides$v.so timeout -k 10 200 python3 - > $O/sides$v.json 2> $O/sides$v.err <<PY || { tail -20 $O/sides$v.err; exit 1; }
import json, time
from indy_plenum_amd import edv, workload
b = workload.DeviceBatch(65536)
args = (b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, 65536, b.d_accept.ptr, 0)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.0:
    edv.time_device(*args, 8)
p, m = edv.profile_device(*args, 20)
print(json.dumps({"sides_mask": $v, "prep_ms": p}))
PY
  cat $O/sides$v.json
done

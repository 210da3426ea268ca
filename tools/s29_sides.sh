#!/bin/bash
# s29: prep kernel time per side at HEAD (EDV_AB_SIDES bit k = run side k:
# 0 hash, 1 A point, 2 R point; measurement builds, their verdicts are
# meaningless), at C2 (65,536) and one 2^18 chunk
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r03/s29; mkdir -p $O; cd $R
for n in 65536 262144; do
for v in 7 1 2 6 3; do
  L=indy-plenum_amd/variants/libedv_sides$v.so
  [ $v = 7 ] && L=indy-plenum_amd/libedv.so
  EDV_ALLOW_MEASUREMENT_LIB=1 EDV_LIB=$R/$L N=$n V=$v timeout -k 10 200 python3 - >> $O/sides.jsonl 2> $O/sides$v.err <<'PY' || { tail -20 $O/sides$v.err; exit 1; }
import json, os, time
from indy_plenum_amd import edv, workload
n = int(os.environ["N"])
b = workload.DeviceBatch(n)
args = (b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr, 0)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.0:
    edv.time_device(*args, 8)
p, m = edv.profile_device(*args, 20)
print(json.dumps({"n": n, "sides_mask": int(os.environ["V"]), "prep_ms": p, "main_ms": m}))
PY
done
done
cat $O/sides.jsonl

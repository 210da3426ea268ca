#!/bin/bash
# Round 4, session 2: min-shard threshold (latency vs n), the synchronous call
# with CU-masked sub-batch streams, and the main kernel's B entries staged
# through the A/R LDS slice (variant breuse) against HEAD, with quick parity.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04/s2; mkdir -p $O; cd $R
fail() { echo "FAILED: $1"; tail -30 "$2"; exit 1; }
timeout -k 10 240 python3 tools/latency_vs_n.py > $O/latency_vs_n.jsonl 2> $O/lat.err || fail lat $O/lat.err
cat $O/latency_vs_n.jsonl
timeout -k 10 240 python3 tools/small_batch_latency.py > $O/small_batch_latency.jsonl 2> $O/sbl.err || fail sbl $O/sbl.err
cat $O/small_batch_latency.jsonl
timeout -k 10 300 python3 tools/e2e_cumask.py > $O/e2e_cumask.jsonl 2> $O/cumask.err || fail cumask $O/cumask.err
tail -1 $O/e2e_cumask.jsonl
EDV_LIB=$R/indy-plenum_amd/variants/libedv_breuse.so EDV_PARITY_QUICK=1 timeout -k 10 400 python3 -u -m pytest \
  tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/parity_breuse.log 2>&1 \
  || fail parity_breuse $O/parity_breuse.log
tail -2 $O/parity_breuse.log
timeout -k 10 500 python3 tools/ab_bench.py indy-plenum_amd/libedv.so indy-plenum_amd/variants/libedv_breuse.so indy-plenum_amd/variants/libedv_breuse_early.so \
  indy-plenum_amd/libedv.so indy-plenum_amd/variants/libedv_breuse.so indy-plenum_amd/variants/libedv_breuse_early.so > $O/ab_breuse.jsonl 2> $O/ab.err \
  || fail ab $O/ab.err
cat $O/ab_breuse.jsonl
export TMPDIR=/tmp
CFGS=1:0,4:0,4:1,1:0:z R=5 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run \
  --output-format csv -- python3 tools/e2e_cumask.py > $O/trace.log 2>&1 || fail trace $O/trace.log
find $O/trace -name "*.csv" | head
python3 tools/trace_overlap.py $O/trace 1:0,4:0,4:1,1:0:z 5 > $O/trace_overlap.json || true
cat $O/trace_overlap.json
echo "session done"

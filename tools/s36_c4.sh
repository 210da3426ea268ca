#!/bin/bash
# C4 (200..4096 B) kernel times and the SHA-256 digest kernel on the current sources
set -o pipefail
O=gpurun_out/r02/s36
mkdir -p $O
timeout -k 10 300 python3 tools/bench_c4.py > $O/c4.jsonl 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
cat $O/c4.jsonl
timeout -k 10 200 python3 tools/bench_digest.py > $O/digest.json 2> $O/digest.err || { tail -20 $O/digest.err; exit 1; }
cat $O/digest.json

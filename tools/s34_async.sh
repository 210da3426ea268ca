#!/bin/bash
# async host path: its GPU tests, then the bench e2e leg
set -o pipefail
O=gpurun_out/r02/s34
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_runtime.py -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "async or host_path or split" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['e2e']))"

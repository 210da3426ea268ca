#!/bin/bash
# split-prep host path: GPU tests of the host path, then the e2e probe
set -o pipefail
O=gpurun_out/r02/s31
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_runtime.py -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "host_split or host_path or multi_device" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python3 tools/e2e_probe.py > $O/e2e_probe.json 2> $O/e2e_probe.err || { tail -20 $O/e2e_probe.err; exit 1; }
cat $O/e2e_probe.json

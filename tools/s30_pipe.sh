mkdir -p gpurun_out/r02/s30
timeout -k 10 200 python3 bench.py --no-e2e --no-cpu-baseline --pipeline > gpurun_out/r02/s30/bench_pipe.json 2>gpurun_out/r02/s30/err1 && \
timeout -k 10 200 python3 bench.py --no-e2e --no-cpu-baseline > gpurun_out/r02/s30/bench_seq.json 2>gpurun_out/r02/s30/err2 && \
python3 - <<'PY'
import json
for f in ["pipe", "seq"]:
    d = json.load(open("gpurun_out/r02/s30/bench_%s.json" % f))
    print(f, d["value"], d["ms_per_step"], d["roofline"]["prep_kernel_ms"], d["roofline"]["main_kernel_ms"])
PY

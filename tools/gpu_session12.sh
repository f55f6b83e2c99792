#!/bin/bash
# GPU-box session 12: UDS round-trip floor vs the plugin's Allocate latency.
set -o pipefail
out=gpurun_out/s12
mkdir -p $out
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || { echo BUILD FAILED; tail -30 $out/build.log; exit 1; }
for bp in 50 0; do
  timeout -k 10 120 build/native/amdgpu-dp-uds-floor --iters 200000 --busy-poll-us $bp | tee -a $out/uds_floor.jsonl || exit 1
done
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json; d=json.load(open('$out/bench.json')); print('bench', d['value'], d['allocate_p99_us'], d['pods_per_s'])"

#!/bin/bash
# GPU-box session 29: 12 interleaved pairs of 1-client busy-poll benches
# (the driver's N=1 shape), native vs nghttp2 HTTP/2 engine.
set -o pipefail
out=gpurun_out/s29
mkdir -p $out
for i in $(seq 1 12); do
  for eng in native nghttp2; do
    DP_HTTP2_SERVER=$eng timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-probe > $out/bench_${eng}_$i.json 2> $out/bench_${eng}_$i.err || { tail -20 $out/bench_${eng}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$out/bench_${eng}_$i.json')); print('P $i $eng', d['value'], d['allocate_p99_us'], d['preferred_p50_us'])"
  done
done

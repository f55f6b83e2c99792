#!/bin/bash
# GPU-box session 25: A/B of the HTTP/2 server engines on one box, interleaved
# (native, nghttp2) x 4, spx-none and auto-mem, 50 steps x 100 pods each.
set -o pipefail
out=${OUT:-gpurun_out/s25}
mkdir -p $out
for i in 1 2 3 4; do
  for eng in native nghttp2; do
    for cfg in spx-none auto-mem; do
      DP_HTTP2_SERVER=$eng timeout -k 10 300 python bench.py --steps 50 --warmup 5 --config $cfg --no-probe > $out/bench_${eng}_${cfg}_$i.json 2> $out/bench_${eng}_${cfg}_$i.err || { tail -20 $out/bench_${eng}_${cfg}_$i.err; exit 1; }
      python -c "import json; d=json.load(open('$out/bench_${eng}_${cfg}_$i.json')); print('$i $eng $cfg', d['value'], d['allocate_p99_us'], d['preferred_p50_us'], d['pods_per_s'])"
    done
  done
done

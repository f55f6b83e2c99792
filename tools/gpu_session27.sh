#!/bin/bash
# GPU-box session 27: larger interleaved A/B of the HTTP/2 engines: bench
# spx-none x 6 each, and the daemon's CPU per RPC (busy-poll off) x 3 each.
set -o pipefail
out=gpurun_out/s27
mkdir -p $out
for i in 1 2 3 4 5 6; do
  for eng in native nghttp2; do
    DP_HTTP2_SERVER=$eng timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-probe > $out/bench_${eng}_$i.json 2> $out/bench_${eng}_$i.err || { tail -20 $out/bench_${eng}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$out/bench_${eng}_$i.json')); print('B $i $eng', d['value'], d['allocate_p99_us'], d['pods_per_s'])"
  done
done
for i in 1 2 3; do
  for eng in native nghttp2; do
    DP_HTTP2_SERVER=$eng timeout -k 10 300 python tools/profile_daemon.py $out/prof_${eng}_$i.txt --busy-poll-us 0 --pods 150000 --real > $out/cpu_${eng}_$i.json 2> $out/cpu_${eng}_$i.err || { tail -20 $out/cpu_${eng}_$i.err; exit 1; }
    echo "C $i $eng $(cat $out/cpu_${eng}_$i.json)"
  done
done

#!/bin/bash
# GPU-box session 40: spread of the driver-shaped headline run (python bench.py,
# defaults) over 10 back-to-back runs on one box.
set -o pipefail
out=${OUT:-gpurun_out/s40}
mkdir -p $out
for i in $(seq 1 10); do
  timeout -k 10 300 python bench.py --no-probe > $out/bench_$i.json 2> $out/bench_$i.err || { tail -5 $out/bench_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$out/bench_$i.json')); print('R $i', d['value'], d['allocate_p99_us'], d['pods_per_s'])"
done

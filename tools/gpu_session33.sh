#!/bin/bash
# GPU-box session 33: placement sensitivity of the 1-client Allocate latency on
# the box's 2 x EPYC 9575F (8-core CCDs, one L3 each). The whole bench (client
# thread + daemon) is confined with taskset; 3 runs per placement.
set -o pipefail
out=gpurun_out/s33
mkdir -p $out
for place in "0,1:same-L3" "0,8:other-L3-same-socket" "0,64:other-socket" "0,128:SMT-siblings" "0-7:one-CCD" "all:unpinned"; do
  cpus=${place%%:*}; name=${place#*:}
  for i in 1 2 3; do
    if [ "$cpus" = all ]; then
      timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-probe > $out/b_${name}_$i.json 2> $out/b_${name}_$i.err || { tail -5 $out/b_${name}_$i.err; exit 1; }
    else
      timeout -k 10 300 taskset -c $cpus python bench.py --steps 20 --warmup 3 --no-probe > $out/b_${name}_$i.json 2> $out/b_${name}_$i.err || { tail -5 $out/b_${name}_$i.err; exit 1; }
    fi
    python -c "import json; d=json.load(open('$out/b_${name}_$i.json')); print('T $name $i', d['value'], d['allocate_p99_us'])"
  done
done

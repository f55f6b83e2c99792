#!/bin/bash
# CONFIGS="spx-none" limits the run to the configs named.
# Allocate() p50 / allocatable curve at 1/2/4/8 GPUs for every BASELINE config on
# the amdsmi mock node model (gloo ranks, no GPU touched) -- the multi-GPU and
# partition configurations the one-GPU box cannot host for real.
set -o pipefail
out=${1:-gpurun_out/curve}
mkdir -p $out
port=29611
for cfg in ${CONFIGS:-spx-none timeslice4 auto-mem cpx-single}; do
  for n in 1 2 4 8; do
    port=$((port + 1))
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $n --steps 20 --warmup 2 --config $cfg --mock --no-probe \
      > $out/$cfg-$n.json 2> $out/$cfg-$n.err || { echo "FAILED $cfg $n"; tail -20 $out/$cfg-$n.err; exit 1; }
    python -c "import json; d=json.loads(open('$out/$cfg-$n.json').read().strip().splitlines()[-1]); print('$cfg', $n, 'allocatable', d['allocatable'], 'p50', d['value'], 'p99', d['allocate_p99_us'], 'pods/s', d['pods_per_s'], 'residency_p50', next(iter((d.get('server_residency') or {}).values()), None) and next(iter(d['server_residency'].values()))['p50_us'])"
  done
done

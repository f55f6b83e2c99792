#!/bin/bash
# GPU-box session 34: --loop-affinity peer-l3 vs none, interleaved x8, 1-client
# bench unpinned (the driver's N=1 shape); then 4/8-rank node model x2 each.
set -o pipefail
out=${OUT:-gpurun_out/s34}
mkdir -p $out
for i in $(seq 1 8); do
  for aff in peer-l3 none; do
    DP_LOOP_AFFINITY=$aff timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-probe > $out/b_${aff}_$i.json 2> $out/b_${aff}_$i.err || { tail -5 $out/b_${aff}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$out/b_${aff}_$i.json')); print('A $aff $i', d['value'], d['allocate_p99_us'])"
  done
done
port=29811
for i in 1 2; do
  for aff in peer-l3 none; do
    for n in 4 8; do
      port=$((port + 1))
      DP_LOOP_AFFINITY=$aff timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $port bench.py --gpus $n --steps 20 --warmup 2 --mock --no-probe > $out/m_${aff}_${n}_$i.json 2> $out/m_${aff}_${n}_$i.err || { tail -5 $out/m_${aff}_${n}_$i.err; exit 1; }
      python -c "import json; d=json.loads(open('$out/m_${aff}_${n}_$i.json').read().strip().splitlines()[-1]); print('M $aff $n $i', d['value'], d['allocate_p99_us'], d['pods_per_s'])"
    done
  done
done

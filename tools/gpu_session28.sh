#!/bin/bash
# GPU-box session 28: HTTP/2 engine A/B with 8 concurrent kubelet clients (the
# driver's N=8 shape) on the 8-GPU node model (gloo ranks, mock amdsmi), x3.
set -o pipefail
out=gpurun_out/s28
mkdir -p $out
port=29711
for i in 1 2 3; do
  for eng in native nghttp2; do
    for n in 4 8; do
      port=$((port + 1))
      DP_HTTP2_SERVER=$eng timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $port bench.py --gpus $n --steps 20 --warmup 2 --mock --no-probe \
        > $out/${eng}_${n}_$i.json 2> $out/${eng}_${n}_$i.err || { echo "FAILED $eng $n"; tail -20 $out/${eng}_${n}_$i.err; exit 1; }
      python -c "import json; d=json.loads(open('$out/${eng}_${n}_$i.json').read().strip().splitlines()[-1]); print('M $i $eng', $n, 'p50', d['value'], 'p99', d['allocate_p99_us'], 'pods/s', d['pods_per_s'])"
    done
  done
done

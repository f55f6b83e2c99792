#!/bin/bash
# GPU-box session 20: client frames batched into one write per request (like
# grpc-go's writer). 1-GPU bench for the three real-hardware configs, the UDS
# floor and the daemon's CPU time per RPC (busy-poll off) next to the floor's.
set -o pipefail
out=${OUT:-gpurun_out/s20}
mkdir -p $out
for cfg in spx-none timeslice4 auto-mem; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --config $cfg > $out/bench_$cfg.json 2> $out/bench_$cfg.err || { tail -20 $out/bench_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('$out/bench_$cfg.json')); print('$cfg', d['allocatable'], d['value'], d['allocate_p99_us'], d['preferred_p50_us'], d['server_allocate_handler_avg_us'], d['pods_per_s'])"
done
for b in 50 0; do
  timeout -k 10 120 build/native/amdgpu-dp-uds-floor --iters 200000 --busy-poll-us $b > $out/floor_bp$b.json || exit 1
  cat $out/floor_bp$b.json
done
timeout -k 10 300 python tools/profile_daemon.py $out/daemon_profile_bp0.txt --busy-poll-us 0 --pods 200000 --real > $out/daemon_cpu_bp0.json 2> $out/daemon_cpu_bp0.err || { tail -20 $out/daemon_cpu_bp0.err; exit 1; }
cat $out/daemon_cpu_bp0.json
head -30 $out/daemon_profile_bp0.txt

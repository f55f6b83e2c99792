#!/bin/bash
# GPU-box session 14: real-hardware table for docs/PERF.md (3 configs) + cold start.
set -o pipefail
out=gpurun_out/s14
mkdir -p $out
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || { echo BUILD FAILED; tail -30 $out/build.log; exit 1; }
for cfg in spx-none timeslice4 auto-mem; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --config $cfg > $out/bench_$cfg.json 2> $out/bench_$cfg.err || { tail -20 $out/bench_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('$out/bench_$cfg.json')); print('$cfg', d['allocatable'], d['value'], d['allocate_p99_us'], d['preferred_p50_us'], d['server_allocate_handler_avg_us'], d['grpcio_client_allocate_p50_us'], d['pods_per_s'])"
done
timeout -k 10 120 python tools/gpu_session2.py daemon > $out/cold.log 2>&1 || { tail -20 $out/cold.log; exit 1; }
cp gpurun_out/s2/cold_start.json $out/ && cat $out/cold_start.json | python -c "import json,sys; d=json.load(sys.stdin); print('cold start register ms', [round(x['register_ms'],1) for x in d])"
tail -3 $out/cold.log

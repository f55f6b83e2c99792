#!/bin/bash
# GPU-box session 38 (end of round 1): GPU suite, smoke, default bench, the three
# real-hardware configs, and rocprofv3 kernel stats of the probe incl. the
# census / interference kernels.
set -o pipefail
out=gpurun_out/s38
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.json 2> $out/smoke.err || { echo SMOKE FAILED; tail -30 $out/smoke.err; exit 1; }
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
cat $out/bench_default.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['allocate_p99_us'], d['pods_per_s'])"
for cfg in spx-none timeslice4 auto-mem; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --config $cfg > $out/bench_$cfg.json 2> $out/bench_$cfg.err || { tail -20 $out/bench_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('$out/bench_$cfg.json')); print('$cfg', d['allocatable'], d['value'], d['allocate_p99_us'], d['preferred_p50_us'], d['server_allocate_handler_avg_us'], d['grpcio_client_allocate_p50_us'], d['pods_per_s'])"
done
cd /tmp
P=$GRAFT_REPO_ROOT/build/probe/amdgpu-dp-probe
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof -o probe -- $P --device 0 --bytes 1073741824 --iters 3 --mfma > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$out/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof_census -o census -- $P --device 0 --census > $GRAFT_REPO_ROOT/$out/prof_census.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$out/prof_census.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof_latency -o latency -- $P --device 0 --latency 500 > $GRAFT_REPO_ROOT/$out/prof_latency.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$out/prof_latency.log; exit 1; }
find $GRAFT_REPO_ROOT/$out -name "*kernel_stats.csv" -exec cat {} \;

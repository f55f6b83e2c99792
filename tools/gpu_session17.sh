#!/bin/bash
# GPU-box session 17 (fresh container rebuild): GPU tests, smoke, 1-GPU bench
# for the three real-hardware configs, probe kernel stats under rocprofv3.
set -o pipefail
out=gpurun_out/s17
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.json 2> $out/smoke.err || { echo SMOKE FAILED; tail -30 $out/smoke.err; exit 1; }
tail -1 $out/smoke.json
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
cat $out/bench_default.json
for cfg in spx-none timeslice4 auto-mem; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --config $cfg > $out/bench_$cfg.json 2> $out/bench_$cfg.err || { tail -20 $out/bench_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('$out/bench_$cfg.json')); print('$cfg', d['allocatable'], d['value'], d['allocate_p99_us'], d['preferred_p50_us'], d['server_allocate_handler_avg_us'], d['grpcio_client_allocate_p50_us'], d['pods_per_s'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof -o probe -- $GRAFT_REPO_ROOT/build/probe/amdgpu-dp-probe --device 0 --bytes 1073741824 --iters 3 --mfma > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$out/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$out/prof -name "*kernel_stats.csv" -exec cat {} \;

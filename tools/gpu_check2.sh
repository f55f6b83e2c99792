#!/bin/bash
# GPU session 2 (see tools/gpu_session2.py). Each GPU step has its own limit.
set -o pipefail
out=gpurun_out/s2
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || { tail -30 $out/build.log; exit 1; }
timeout -k 10 300 python tools/gpu_session2.py sweep > $out/sweep.log 2>&1 || { tail -20 $out/sweep.log; exit 1; }
tail -3 $out/sweep.log
timeout -k 10 300 python tools/gpu_session2.py daemon > $out/daemon.log 2>&1 || { tail -20 $out/daemon.log; exit 1; }
tail -2 $out/daemon.log
for cfg in spx-none timeslice4 auto-mem; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --config $cfg > $out/bench_$cfg.json 2> $out/bench_$cfg.err || { tail -20 $out/bench_$cfg.err; exit 1; }
  cut -c1-400 $out/bench_$cfg.json
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof -o probe -- python3 $GRAFT_REPO_ROOT/tools/probe_once.py > $GRAFT_REPO_ROOT/$out/rocprof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/rocprof.log; exit 1; }
find $GRAFT_REPO_ROOT/$out/prof -name "*.csv" | head
echo session2 done

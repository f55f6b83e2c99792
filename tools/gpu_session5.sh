#!/bin/bash
# GPU-box session 5: GPU tests, smoke, 1-GPU bench (multi-loop server), concurrent
# client scaling (1 vs 8 loops), rocprof kernel stats of the HIP probe.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
out=gpurun_out/s5
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || { echo BUILD FAILED; tail -30 $out/build.log; exit 1; }
echo built
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $out/pytest_gpu.log 2>&1; rc=$?
tail -15 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python __graft_entry__.py smoke > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 2 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
# CPU-only (mock node model): concurrency scaling of one plugin socket.
timeout -k 10 300 python tools/concurrency.py --server-threads 1 > $out/conc_1loop.json 2> $out/conc_1loop.err || { tail -20 $out/conc_1loop.err; exit 1; }
timeout -k 10 300 python tools/concurrency.py > $out/conc_default.json 2> $out/conc_default.err || { tail -20 $out/conc_default.err; exit 1; }
cat $out/conc_1loop.json $out/conc_default.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof -o probe -- python3 $GRAFT_REPO_ROOT/tools/probe_once.py > $GRAFT_REPO_ROOT/$out/rocprof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/rocprof.log; exit 1; }
echo rocprof done

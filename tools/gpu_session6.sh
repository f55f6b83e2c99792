#!/bin/bash
# GPU-box session 6: busy-poll A/B (bench at 0 vs default 50 us), GPU tests, smoke.
set -o pipefail
out=gpurun_out/s6
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || { echo BUILD FAILED; tail -30 $out/build.log; exit 1; }
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $out/pytest_gpu.log 2>&1; rc=$?
tail -3 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python __graft_entry__.py smoke > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $out/bench_default.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
DP_BUSY_POLL_US=0 timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $out/bench_nospin.json 2> $out/bench0.err || { tail -20 $out/bench0.err; exit 1; }
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $out/bench_default2.json 2> $out/bench2.err || { tail -20 $out/bench2.err; exit 1; }
for f in bench_default bench_nospin bench_default2; do python -c "import json,sys; d=json.load(open('$out/$f.json')); print('$f', d['value'], d['allocate_p99_us'], d['pods_per_s'])"; done
timeout -k 10 300 python tools/concurrency.py --busy-poll-us 0 > $out/conc_nospin.json 2> $out/conc0.err || { tail -20 $out/conc0.err; exit 1; }
timeout -k 10 300 python tools/concurrency.py > $out/conc_default.json 2> $out/conc.err || { tail -20 $out/conc.err; exit 1; }
cat $out/conc_nospin.json $out/conc_default.json

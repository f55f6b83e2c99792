#!/bin/bash
# GPU-box session 10: GPU tests (labels), bench, concurrency.
set -o pipefail
out=gpurun_out/s10
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || { echo BUILD FAILED; tail -30 $out/build.log; exit 1; }
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $out/pytest_gpu.log 2>&1; rc=$?
tail -3 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python __graft_entry__.py smoke > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json; d=json.load(open('$out/bench.json')); print('bench', d['value'], d['allocate_p99_us'], d['pods_per_s'])"
timeout -k 10 300 python tools/concurrency.py > $out/conc.json 2> $out/conc.err || { tail -20 $out/conc.err; exit 1; }
cat $out/conc.json

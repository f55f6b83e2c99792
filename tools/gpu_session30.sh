#!/bin/bash
# GPU-box session 30: GPU suite + smoke on the native HTTP/2 engine, default
# bench, then the 1/2/4/8-rank node-model curve for every BASELINE config.
set -o pipefail
out=gpurun_out/s30
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.json 2> $out/smoke.err || { echo SMOKE FAILED; tail -30 $out/smoke.err; exit 1; }
tail -1 $out/smoke.json
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$out/bench_default.json')); print('default', d['value'], d['allocate_p99_us'], d['pods_per_s'])"
bash tools/mock_curve.sh $out/curve

#!/bin/bash
# GPU-box session 23: full GPU suite (incl. the CU-share isolation test) + smoke.
set -o pipefail
out=gpurun_out/s23
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $out/pytest_gpu.log; exit 1; }
tail -4 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.json 2> $out/smoke.err || { echo SMOKE FAILED; tail -30 $out/smoke.err; exit 1; }
tail -1 $out/smoke.json

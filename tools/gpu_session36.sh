#!/bin/bash
# GPU-box session 36: 5-minute soak on the native HTTP/2 engine with real
# libamd_smi (4 churn clients, SIGHUP restarts, kubelet restarts, scrapes,
# RSS/fd/thread sampling), then the GPU suite once more.
set -o pipefail
out=gpurun_out/s36
mkdir -p $out
timeout -k 10 420 python -u tools/soak.py --seconds 300 --clients 4 --real --out $out/soak_real.json > $out/soak.log 2>&1 || { tail -30 $out/soak.log; exit 1; }
tail -5 $out/soak.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log

#!/bin/bash
# GPU-box session 13: 5-minute soak on real libamd_smi, then 2 minutes on the 8-GPU node model.
set -o pipefail
out=gpurun_out/s13
mkdir -p $out
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || { echo BUILD FAILED; tail -30 $out/build.log; exit 1; }
timeout -k 10 420 python tools/soak.py --seconds 300 --clients 4 --real --out $out/soak_real.json || exit 1
timeout -k 10 240 python tools/soak.py --seconds 120 --clients 8 --out $out/soak_mock8.json || exit 1

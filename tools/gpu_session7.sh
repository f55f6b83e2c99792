#!/bin/bash
# GPU-box session 7: GPU tests (memory-grant cap), copy-kernel sweep (nt loads,
# chunked), daemon CPU profile under churn on the real GPU.
set -o pipefail
out=gpurun_out/s7
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || { echo BUILD FAILED; tail -30 $out/build.log; exit 1; }
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $out/pytest_gpu.log 2>&1; rc=$?
tail -5 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "
import json
from k8s_gpu_sharing_plugin_amd.ops import probe
for nb in (1 << 30, 2 << 30):
    r = probe.bw_sweep(0, nb, 10)
    r.sort(key=lambda x: -x['gbps'])
    print(nb >> 20, 'MiB top5', json.dumps(r[:5]))
    json.dump(r, open('$out/sweep_%dmib.json' % (nb >> 20), 'w'), indent=1)
" > $out/sweep.log 2>&1 || { tail -20 $out/sweep.log; exit 1; }
cat $out/sweep.log
timeout -k 10 300 python tools/profile_daemon.py $out/daemon_profile_real.txt --real > $out/profile.log 2>&1 || { tail -20 $out/profile.log; exit 1; }
cat $out/profile.log; head -30 $out/daemon_profile_real.txt

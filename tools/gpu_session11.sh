#!/bin/bash
# GPU-box session 11: MFMA probe + GPU tests + rocprof kernel stats of the probe kernels.
set -o pipefail
out=gpurun_out/s11
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || { echo BUILD FAILED; tail -30 $out/build.log; exit 1; }
timeout -k 10 120 python -c "
import json
from k8s_gpu_sharing_plugin_amd.ops import probe
for it in (1 << 12, 1 << 14, 1 << 16):
    print(json.dumps(probe.mfma(0, it)))
" > $out/mfma.log 2>&1; rc=$?
cat $out/mfma.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $out/pytest_gpu.log 2>&1; rc=$?
tail -3 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof -o probe -- $GRAFT_REPO_ROOT/build/probe/amdgpu-dp-probe --device 0 --bytes 1073741824 --iters 10 --mfma > $GRAFT_REPO_ROOT/$out/rocprof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/rocprof.log; exit 1; }
cat $GRAFT_REPO_ROOT/$out/prof/probe_kernel_stats.csv | cut -c1-160

#!/bin/bash
# GPU-box session 19: CU-partitioned replicas end to end (daemon on real
# libamd_smi -> HSA_CU_MASK -> census), HSA_CU_MASK multi-device syntax check,
# then the full GPU suite.
set -o pipefail
out=gpurun_out/s19
mkdir -p $out
P=build/probe/amdgpu-dp-probe
# ';'-separated per-device entries: device 0 must get bits 64-127 whichever order
for m in "0:64-127;1:0-31" "1:0-31;0:64-127"; do
  HSA_CU_MASK="$m" timeout -k 5 60 $P --device 0 --census > $out/census_multi.json 2> $out/census_multi.err || { cat $out/census_multi.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/census_multi.json')); print(repr('$m'), 'seen', d['cus_seen'], 'per_xcc', d['per_xcc'])"
done
timeout -k 10 300 build/native/amdgpu-device-plugin --dry-run --devices 0 --resource-config gpu:sharedgpu:4 --replica-cu-mask > $out/dry_run.json 2> $out/dry_run.err || { cat $out/dry_run.err; exit 1; }
cat $out/dry_run.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log

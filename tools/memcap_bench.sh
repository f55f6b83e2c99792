#!/bin/bash
# Allocation-path cost of the HBM-cap shim on the GPU box: the same HIP program
# without the shim, with it but no cap, and with a 4000 MiB cap, interleaved
# over 3 rounds (the shim is appended to whatever the environment preloads).
set -eo pipefail
out=${OUT:-gpurun_out/memcap_bench}
mkdir -p "$out"
B=build/probe/amdgpu-dp-memcap-bench
SHIM=$PWD/build/native/libadp_memcap.so
PRE="${LD_PRELOAD:+$LD_PRELOAD }$SHIM"
: > $out/runs.jsonl
for round in 1 2 3; do
  timeout -k 5 120 $B 20000 >> $out/runs.jsonl
  LD_PRELOAD="$PRE" timeout -k 5 120 $B 20000 >> $out/runs.jsonl
  LD_PRELOAD="$PRE" AMD_GPU_MEMORY_LIMIT_MIB=4000 ADP_MEMCAP_KEY=bench-$$ timeout -k 5 120 $B 20000 >> $out/runs.jsonl
done
rm -f /dev/shm/adp-memcap-key-bench-$$-*
cat $out/runs.jsonl

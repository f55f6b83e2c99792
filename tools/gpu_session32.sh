#!/bin/bash
# GPU-box session 32: where does the N=1 bimodality come from? CPU topology,
# then the 1-client bench pinned (client + daemon) to CPUs sharing an L3,
# CPUs on different L3s, and unpinned.
set -o pipefail
out=gpurun_out/s32
mkdir -p $out
lscpu > $out/lscpu.txt; lscpu -e=CPU,CORE,SOCKET,NODE,CACHE > $out/lscpu_e.txt 2>/dev/null || true
head -20 $out/lscpu.txt
grep -E "^ *(0|1|2|3|4|5|6|7|8|9|10|11|12|13|14|15|16|17) " $out/lscpu_e.txt | head -20
cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null || cat /sys/fs/cgroup/cpuset/cpuset.cpus 2>/dev/null || true
python3 -c "import os; print('affinity', sorted(os.sched_getaffinity(0))[:64], len(os.sched_getaffinity(0)))"

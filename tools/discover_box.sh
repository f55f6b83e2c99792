#!/bin/bash
# Hardware discovery on the MI355X box: what amdsmi / sysfs / devnodes look like
# unprivileged. Output is used to shape the real-hardware fixture + tests.
out=gpurun_out/discover
mkdir -p $out
id > $out/id.txt 2>&1
ls -la /dev/kfd /dev/dri > $out/devnodes.txt 2>&1
timeout -k 5 60 amd-smi list > $out/amdsmi_list.txt 2>&1
timeout -k 5 60 amd-smi static > $out/amdsmi_static.txt 2>&1
timeout -k 5 60 amd-smi topology > $out/amdsmi_topology.txt 2>&1
timeout -k 5 60 amd-smi partition > $out/amdsmi_partition.txt 2>&1
for d in /sys/class/drm/card*/device; do echo "== $d"; cat $d/current_compute_partition $d/current_memory_partition $d/available_compute_partition $d/numa_node 2>&1; done > $out/sysfs.txt 2>&1
ls /sys/class/kfd/kfd/topology/nodes > $out/kfd_nodes.txt 2>&1
nproc > $out/nproc.txt
timeout -k 5 60 rocminfo > $out/rocminfo.txt 2>&1
echo done

#!/usr/bin/env python3
"""The CPUs this process may run on, grouped by L3 (CCD) and NUMA node, as JSON:
what decides whether a client and a gRPC loop can share an L3 (docs/PERF.md
"CPU placement")."""

import json
import os


def _cpulist(text):
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def main():
    allowed = sorted(os.sched_getaffinity(0))
    l3, numa = {}, {}
    for c in allowed:
        base = f"/sys/devices/system/cpu/cpu{c}"
        key = _read(f"{base}/cache/index3/shared_cpu_list") or "?"
        l3.setdefault(key, []).append(c)
        node = next((d for d in os.listdir(base) if d.startswith("node") and d[4:].isdigit()), "node?")
        numa.setdefault(node, []).append(c)
    print(json.dumps({
        "online": _read("/sys/devices/system/cpu/online"),
        "allowed": len(allowed),
        "cgroup_cpuset": _read("/sys/fs/cgroup/cpuset.cpus.effective"),
        "cpu_max": _read("/sys/fs/cgroup/cpu.max"),
        "l3_groups_used": len(l3),
        "allowed_per_l3": {k: v for k, v in l3.items()},
        "allowed_per_numa": {k: len(v) for k, v in numa.items()},
        "smt_siblings_cpu0": _read(f"/sys/devices/system/cpu/cpu{allowed[0]}/topology/thread_siblings_list"),
    }, indent=1))


if __name__ == "__main__":
    main()

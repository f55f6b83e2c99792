#!/usr/bin/env python3
"""Side by side: which amdsmi queries and device nodes still work when a device
cgroup denies the device nodes (reports from `amdgpu-device-plugin --smi-report`,
first = unrestricted). Prints one row per query: status per report."""
import json
import sys


def load(path):
    try:
        return json.load(open(path))
    except (OSError, ValueError) as e:
        return {"error": str(e)}


def main(paths):
    reps = [load(p) for p in paths]
    names = [p.rsplit("/", 1)[-1].replace("smi_report", "").strip("_.json") or "unrestricted" for p in paths]
    print("query".ljust(32) + "".join(n[:14].ljust(16) for n in names))
    first = reps[0].get("processors") or [{}]
    for q in first[0]:
        row = q.ljust(32)
        for r in reps:
            procs = r.get("processors") or [{}]
            v = procs[0].get(q, {})
            row += str(v.get("status", "-")).ljust(16)
        print(row)
    for r, n in zip(reps, names):
        denied = [a["node"] for a in r.get("device_access", []) if a.get("errno")]
        print(f"{n}: enumeration {r.get('enumeration')}, nodes denied: {denied or 'none'}")


if __name__ == "__main__":
    main(sys.argv[1:])

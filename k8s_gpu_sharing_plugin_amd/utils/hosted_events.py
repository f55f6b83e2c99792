"""Real KFD events through the daemon's own code, on a box without root.

KFD delivers an unprivileged event registration only the per-process events
of its own process (measured on the MI355X: profiles/r6/raw_events*.json --
a PROCESS_START of the registering process arrives, another process's never
does), so this helper process hosts the monitor or the relay (libadp_capi)
and then opens the GPU itself through HIP:

    python -m k8s_gpu_sharing_plugin_amd.utils.hosted_events monitor
        the in-process monitor with --health-event-extra-types 12,13; prints one
        JSON line: what it counted (amdgpu_dp_gpu_events_total's source) and
        whether health changed;
    python -m k8s_gpu_sharing_plugin_amd.utils.hosted_events relay <socket>
        the event relay on <socket>; prints "ready", waits for a line on stdin,
        opens the GPU, prints "opened" and a JSON line, waits for another line,
        stops the relay (tests/test_gpu_events.py runs the daemon against it).

Only for the GPU tests: the daemon itself never opens a GPU.
"""

import ctypes
import json
import sys
import time

from . import native


def open_gpu() -> dict:
    """hipInit, hipSetDevice(0), hipMalloc, hipDeviceSynchronize, hipFree in this
    process; `hipInit_wall` is hipInit's [start, end] on the wall clock the
    daemon's and the relay's log lines carry (KFD's PROCESS_START comes from it)."""
    for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
        try:
            hip = ctypes.CDLL(name)
            break
        except OSError:
            hip = None
    if hip is None:
        return {"error": "libamdhip64.so not found"}
    t = time.time()
    out = {"hipInit": hip.hipInit(0)}
    out["hipInit_wall"] = [t, time.time()]
    if out["hipInit"] == 0:
        out["hipSetDevice"] = hip.hipSetDevice(0)
        p = ctypes.c_void_p()
        out["hipMalloc"] = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(64 << 20))
        out["hipDeviceSynchronize"] = hip.hipDeviceSynchronize()
        out["hipFree"] = hip.hipFree(p) if p.value else -1
    return out


def run_monitor() -> int:
    m = native.HostedMonitor(extra_types="12,13")
    try:
        time.sleep(0.5)  # registered, first poll
        before = m.state()
        hip = open_gpu()
        deadline = time.monotonic() + 10
        st = m.state()
        while time.monotonic() < deadline and not any(e["type"] == "PROCESS_START" for e in st["events"]):
            time.sleep(0.1)
            st = m.state()
        time.sleep(0.5)
        st = m.state()
        print(json.dumps({"before": before, "hip": hip, "after": st}), flush=True)
    finally:
        m.close()
    return 0


def run_relay(socket_path: str) -> int:
    r = native.HostedRelay(socket_path, extra_types="12,13")
    try:
        print("ready", flush=True)
        sys.stdin.readline()
        hip = open_gpu()
        print("opened", flush=True)
        print(json.dumps({"hip": hip}), flush=True)
        sys.stdin.readline()
    finally:
        rc = r.close()
    return rc


if __name__ == "__main__":
    if sys.argv[1:2] == ["monitor"]:
        sys.exit(run_monitor())
    if sys.argv[1:2] == ["relay"] and len(sys.argv) == 3:
        sys.exit(run_relay(sys.argv[2]))
    sys.exit(__doc__)

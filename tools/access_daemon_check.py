#!/usr/bin/env python3
"""The daemon on real libamd_smi with the device nodes denied (EPERM, as a
device cgroup does): does it enumerate, register, poll health, and does its
log name the cause of events being off? Writes the daemon log to argv[1]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_sharing_plugin_amd import BUILD_DIR  # noqa: E402
from k8s_gpu_sharing_plugin_amd.utils import harness  # noqa: E402


def main(log_out, allow=""):
    d = harness.scratch_dir("adpacc")
    kub = harness.NativeKubelet(os.path.join(d, "kubelet.sock")).start()
    env = {"LD_PRELOAD": os.path.join(BUILD_DIR, "libadp_devcgroup_sim.so"), "DP_HEALTH_POLL_MS": "500"}
    if allow:
        env["ADP_DEVCGROUP_ALLOW"] = allow
    daemon = harness.Daemon(d, real_smi=True, env=env).start()
    res = {}
    try:
        reg = kub.wait(lambda e: e.get("event") == "register", 30)
        devs = kub.wait(lambda e: e.get("event") == "devices", 30)
        res = {"registered": reg.get("resource"), "healthy": devs.get("healthy"), "total": devs.get("total")}
        daemon.wait_log("health poll #1", timeout=20)
    finally:
        daemon.stop()
        kub.stop()
        with open(log_out, "w") as f:
            f.write(daemon.log())
    log = open(log_out).read()
    res["events_line"] = [ln for ln in log.splitlines() if "events off" in ln or "health monitor watching" in ln]
    res["access_line"] = [ln for ln in log.splitlines() if "device access" in ln]
    res["poll_line"] = [ln for ln in log.splitlines() if "health poll #1" in ln]
    print(res)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")

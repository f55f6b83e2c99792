#!/usr/bin/env python3
"""What the DaemonSet costs a node while nobody admits pods: the daemon with
its production defaults (health events + polling, /metrics scraped every
--scrape-s like a ServiceMonitor, optionally --enforce-memory-units with the
driver-side HBM check) registered with a stub kubelet, left idle for
--seconds. Reports CPU time per second (user + system, all threads), context
switches per second (all threads: every wake-up the daemon causes), RSS,
threads and fds, from /proc.

  python tools/idle_footprint.py [--real] [--enforce] [--relay] [--seconds 60] [--scrape-s 15]

--relay: the chart's layout -- an event relay process next to the daemon, which
takes its events (and, with --enforce, its driver-side scans) from it; the
relay's own CPU, wake-ups and RSS are reported under "relay".

Prints one JSON object.
"""
import argparse
import glob
import json
import os
import socket
import sys
import time
import urllib.request

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_sharing_plugin_amd.models import fixtures  # noqa: E402
from k8s_gpu_sharing_plugin_amd.utils import harness  # noqa: E402


def cpu_seconds(pid):
    """user + system CPU of the whole process (all threads), seconds."""
    with open(f"/proc/{pid}/stat") as f:
        fields = f.read().rsplit(")", 1)[1].split()
    tick = os.sysconf("SC_CLK_TCK")
    return (int(fields[11]) + int(fields[12])) / tick  # utime, stime


def context_switches(pid):
    """Voluntary + involuntary context switches summed over the threads."""
    total = 0
    for status in glob.glob(f"/proc/{pid}/task/*/status"):
        try:
            with open(status) as f:
                for line in f:
                    if line.startswith(("voluntary_ctxt_switches:", "nonvoluntary_ctxt_switches:")):
                        total += int(line.split()[1])
        except OSError:  # a thread that just exited
            pass
    return total


def proc_stats(pid):
    out = {"fds": len(os.listdir(f"/proc/{pid}/fd"))}
    with open(f"/proc/{pid}/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                out["rss_mib"] = round(int(line.split()[1]) / 1024, 1)
            elif line.startswith("Threads:"):
                out["threads"] = int(line.split()[1])
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--real", action="store_true", help="real libamd_smi (a GPU box)")
    ap.add_argument("--enforce", action="store_true", help="memory units with --enforce-memory-units")
    ap.add_argument("--seconds", type=float, default=60)
    ap.add_argument("--scrape-s", type=float, default=15)
    ap.add_argument("--settle-s", type=float, default=3, help="idle time before measuring (start-up excluded)")
    ap.add_argument("--relay", action="store_true", help="events and scans through an event relay process")
    a = ap.parse_args(argv)
    d = harness.scratch_dir("adpidle")
    kub = harness.NativeKubelet(os.path.join(d, "kubelet.sock")).start()
    with socket.socket() as s0:
        s0.bind(("127.0.0.1", 0))
        port = s0.getsockname()[1]
    args = ["--metrics-addr", f"127.0.0.1:{port}", "--health-state-file", os.path.join(d, "health.state")]
    if a.real:
        args += ["--devices", "0"]
    if a.enforce:
        from k8s_gpu_sharing_plugin_amd import BUILD_DIR
        args += ["--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units",
                 "--memcap-lib", os.path.join(BUILD_DIR, "libadp_memcap.so")]
    fx = None if a.real else dict(fixtures.node(8), events_open_kfd=True)
    relay = None
    if a.relay:
        esock = os.path.join(d + ".relay", "events.sock")
        os.makedirs(os.path.dirname(esock), exist_ok=True)
        relay = harness.Daemon(d + ".relay", fx, args=["--event-relay", "--health-event-socket", esock],
                               real_smi=a.real, env={"ADP_LOG_LEVEL": "warn"}).start()
        deadline = time.time() + 30
        while not os.path.exists(esock):
            if time.time() > deadline or relay.proc.poll() is not None:
                raise SystemExit("the relay never listened:\n" + relay.log()[-3000:])
            time.sleep(0.05)
        args += ["--health-event-socket", esock]
    # production defaults: no DP_HEALTH_POLL_MS / DP_DRIVER_HBM_POLL_MS overrides
    dm = harness.Daemon(d, fx, args=args, real_smi=a.real, env={"ADP_LOG_LEVEL": "warn"}).start()
    try:
        if kub.wait(lambda e: e.get("event") == "devices", 30) is None:
            raise SystemExit("the daemon never delivered a device list:\n" + dm.log()[-3000:])
        time.sleep(a.settle_s)
        pid = dm.proc.pid
        rpid = relay.proc.pid if relay else None
        c0, s0_, t0 = cpu_seconds(pid), context_switches(pid), time.monotonic()
        rc0, rs0 = (cpu_seconds(rpid), context_switches(rpid)) if rpid else (0, 0)
        scrapes, next_scrape, t_end = 0, t0, t0 + a.seconds
        while time.monotonic() < t_end:
            if time.monotonic() >= next_scrape:
                with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
                    r.read()
                scrapes += 1
                next_scrape += a.scrape_s
            time.sleep(min(0.5, max(0.0, t_end - time.monotonic())))
        dt = time.monotonic() - t0
        c1, s1 = cpu_seconds(pid), context_switches(pid)
        res = {"real_smi": a.real, "enforce": a.enforce, "seconds": round(dt, 1), "scrapes": scrapes,
               "cpu_ms_per_s": round((c1 - c0) * 1e3 / dt, 3),
               "cpu_pct_of_a_core": round((c1 - c0) * 100 / dt, 3),
               "context_switches_per_s": round((s1 - s0_) / dt, 1), **proc_stats(pid),
               "daemon_alive": dm.proc.poll() is None}
        if rpid:
            rc1, rs1 = cpu_seconds(rpid), context_switches(rpid)
            res["relay"] = {"cpu_pct_of_a_core": round((rc1 - rc0) * 100 / dt, 3),
                            "context_switches_per_s": round((rs1 - rs0) / dt, 1), **proc_stats(rpid),
                            "alive": relay.proc.poll() is None}
    finally:
        code = dm.stop()
        kub.stop()
        if relay and relay.proc.poll() is None:
            relay.stop()
    res["daemon_exit"] = code
    print(json.dumps(res), flush=True)
    return 0 if res["daemon_alive"] and code in (0, None) else 1


if __name__ == "__main__":
    sys.exit(main())

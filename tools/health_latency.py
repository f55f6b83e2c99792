#!/usr/bin/env python3
"""How fast a GPU failure reaches the scheduler: an amdsmi GPU_PRE_RESET event
(the mock's event FIFO) until the kubelet (the native stub, on the same
CLOCK_MONOTONIC) receives the device list with that GPU Unhealthy, and
GPU_POST_RESET until it is Healthy again. The daemon under test runs its
production defaults (events on, health polling every 5 s), so what is timed
is the event path: amdsmi wait -> ledger -> every affected plugin's
ListAndWatch.

  python tools/health_latency.py [--rounds 20] [--gpus 8] [--resource-config gpu:sharedgpu:4] [--relay]

--relay: the event goes through an event relay process (the chart's layout):
amdsmi wait in the relay -> relay socket -> the daemon's monitor -> ListAndWatch.

Prints one JSON object (median / max in ms per transition).
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_sharing_plugin_amd.models import fixtures  # noqa: E402
from k8s_gpu_sharing_plugin_amd.utils import harness  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--resource-config", default="gpu:sharedgpu:4")
    ap.add_argument("--relay", action="store_true")
    a = ap.parse_args(argv)
    d = harness.scratch_dir("adphl")
    fifo = os.path.join(d + ".fixture", "events")
    os.makedirs(os.path.dirname(fifo), exist_ok=True)
    os.mkfifo(fifo)
    kub = harness.NativeKubelet(os.path.join(d, "kubelet.sock")).start()
    fx = dict(fixtures.node(a.gpus), events_open_kfd=True)
    relay = None
    args = ["--resource-config", a.resource_config]
    if a.relay:
        sock = os.path.join(d + ".fixture", "events.sock")
        relay = harness.Daemon(d + ".relay", fx, args=["--event-relay", "--health-event-socket", sock],
                               event_fifo=fifo).start()
        relay.wait_log("relaying amdsmi events on", timeout=30)
        args += ["--health-event-socket", sock]
    dm = harness.Daemon(d, fx, args=args, event_fifo=None if a.relay else fifo).start()
    down, up = [], []
    try:
        first = kub.wait(lambda e: e.get("event") == "devices", 30)
        total = first["total"]
        dm.wait_log("events on through the relay" if a.relay else "health monitor watching", timeout=30)
        fd = os.open(fifo, os.O_WRONLY)
        try:
            for r in range(a.rounds):
                gpu = r % a.gpus
                # mock event line: "<gpu> <amdsmi event type> <message>"
                for code, want, out in ((3, lambda h: h < total, down),    # GPU_PRE_RESET
                                        (4, lambda h: h == total, up)):    # GPU_POST_RESET
                    mark = len(kub.events)
                    t0 = time.monotonic()
                    os.write(fd, f"{gpu} {code} reset\n".encode())
                    e = kub.wait(lambda e: e.get("event") == "devices" and want(e["healthy"]), 10, since=mark)
                    out.append((e["t_us"] / 1e6 - t0) * 1e3)
        finally:
            os.close(fd)
    finally:
        dm.stop()
        kub.stop()
        if relay:
            relay.stop()

    def summary(xs):
        return {"median_ms": round(statistics.median(xs), 3), "max_ms": round(max(xs), 3), "n": len(xs)}

    res = {"gpus": a.gpus, "resource_config": a.resource_config, "advertised": total, "relay": a.relay,
           "event_to_unhealthy": summary(down), "event_to_healthy": summary(up)}
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

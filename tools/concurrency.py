"""Concurrent-client scaling of one plugin socket.

One daemon (amdsmi mock, N-GPU node model) serves 1/2/4/8 native kubelet-stub
bench clients at once; each client churns pods (GetPreferredAllocation +
Allocate) over its own share of the devices. Prints one JSON object with the
per-concurrency p50/p99 Allocate latency and aggregate pods/s. This is the load
shape of the driver's multi-GPU bench (one client per GPU rank against one
daemon) and shows what the multi-loop server buys.

  python tools/concurrency.py [--gpus 8] [--pods 4000] [--server-threads 0] [--busy-poll-us N]
"""

import argparse
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_sharing_plugin_amd import KUBELET_STUB  # noqa: E402
from k8s_gpu_sharing_plugin_amd.models import fixtures  # noqa: E402
from k8s_gpu_sharing_plugin_amd.utils import harness  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--pods", type=int, default=4000)
    ap.add_argument("--clients", default="1,2,4,8")
    ap.add_argument("--server-threads", type=int, default=0)
    ap.add_argument("--busy-poll-us", type=int, default=None)
    a = ap.parse_args()
    d = harness.scratch_dir("adpconc")
    k = harness.NativeKubelet(os.path.join(d, "kubelet.sock")).start()
    args = ["--server-threads", str(a.server_threads)] if a.server_threads else []
    if a.busy_poll_us is not None:
        args += ["--busy-poll-us", str(a.busy_poll_us)]
    dm = harness.Daemon(d, fixtures.node(a.gpus), args=args,
                        env={"ADP_LOG_LEVEL": "warn", "DP_HEALTH_POLL_MS": "0"}).start()
    out = {"gpus": a.gpus, "pods_per_client": a.pods, "server_threads": a.server_threads or "default",
           "busy_poll_us": "default" if a.busy_poll_us is None else a.busy_poll_us, "runs": []}
    try:
        reg = k.wait(lambda e: e.get("event") == "register", 20)
        sock = os.path.join(d, reg["endpoint"])
        for n in (int(x) for x in a.clients.split(",")):
            procs = [subprocess.Popen([KUBELET_STUB, "bench", "--socket", sock, "--pods", str(a.pods),
                                       "--warmup", "500", "--rank", str(r), "--world", str(n)],
                                      stdout=subprocess.PIPE, text=True) for r in range(n)]
            res = [json.loads(p.communicate(timeout=300)[0]) for p in procs]
            run = {"clients": n,
                   "allocate_p50_us_max": max(r["allocate"]["p50_us"] for r in res),
                   "allocate_p99_us_max": max(r["allocate"]["p99_us"] for r in res),
                   "pods_per_s_total": round(sum(r["pods_per_s"] for r in res))}
            out["runs"].append(run)
            print(json.dumps(run), file=sys.stderr, flush=True)
    finally:
        dm.stop()
        k.stop()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Placement diagnosis for the 1-client bench: where the client thread runs at
connect time and after the churn, which L3 the serving loop followed, and the
Allocate p50 -- to see what the slow runs have in common.

  python tools/diag_placement.py [--runs 8] [--pods 3000]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_sharing_plugin_amd.utils import harness, native  # noqa: E402


def cpu_now():
    with open("/proc/thread-self/stat") as f:
        return int(f.read().rsplit(")", 1)[1].split()[36])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=8)
    ap.add_argument("--pods", type=int, default=3000)
    ap.add_argument("--mock", action="store_true")
    ap.add_argument("--init-hip", action="store_true", help="initialise HIP in the client process first (as bench.py does)")
    a = ap.parse_args()
    if a.init_hip:
        import torch
        torch.cuda.is_available()
        torch.cuda.synchronize()
    for i in range(a.runs):
        d = harness.scratch_dir("adpdiag")
        k = harness.NativeKubelet(os.path.join(d, "kubelet.sock")).start()
        fx = None
        if a.mock:
            from k8s_gpu_sharing_plugin_amd.models import fixtures
            fx = fixtures.node(1)
        dm = harness.Daemon(d, fx, real_smi=not a.mock, args=["--devices", "0"],
                            env={"DP_HEALTH_POLL_MS": "0", "ADP_LOG_LEVEL": os.environ.get("DIAG_LOG_LEVEL", "debug")}).start()
        try:
            reg = k.wait(lambda e: e.get("event") == "register", 30)
            c0 = cpu_now()
            cl = native.ChurnClient(os.path.join(d, reg["endpoint"]))
            c1 = cpu_now()
            cl.run(500)
            cl.run(a.pods)
            c2 = cpu_now()
            st = cl.stats()
            cl.close()
            follow = [ln.split("grpc-server: ", 1)[1] for ln in dm.log().splitlines() if "served from its L3" in ln]
            print(json.dumps({"run": i, "p50_us": st["allocate"]["p50_us"], "client_cpu": [c0, c1, c2],
                              "follow": follow}), flush=True)
        finally:
            dm.stop()
            k.stop()


if __name__ == "__main__":
    main()

"""CPU profile of the daemon under pod churn (built-in sampler, ADP_PROFILE_OUT).

  python tools/profile_daemon.py OUT.txt [--busy-poll-us N] [--pods 50000] [--real]

One native stub-kubelet client churns pods (GetPreferredAllocation + Allocate)
against one daemon (1-GPU mock node, or the real GPU with --real); the daemon
samples its own PCs on a CPU-time timer and writes a flat profile at exit.
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


def _cpu_s(pid):
    """utime + stime of a process, in seconds (/proc/<pid>/stat fields 14 and 15)."""
    with open(f"/proc/{pid}/stat") as f:
        fields = f.read().rsplit(")", 1)[1].split()
    return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--busy-poll-us", default=None)
    ap.add_argument("--pods", type=int, default=50000)
    ap.add_argument("--real", action="store_true")
    a = ap.parse_args()
    d = harness.scratch_dir("adpprof")
    k = harness.NativeKubelet(os.path.join(d, "kubelet.sock")).start()
    args = ["--server-threads", "1", "--devices", "0"]
    if a.busy_poll_us is not None:
        args += ["--busy-poll-us", str(a.busy_poll_us)]
    dm = harness.Daemon(d, None if a.real else fixtures.node(1), args=args, real_smi=a.real,
                        env={"ADP_LOG_LEVEL": "warn", "DP_HEALTH_POLL_MS": "0",
                             "ADP_PROFILE_OUT": os.path.abspath(a.out)}).start()
    try:
        reg = k.wait(lambda e: e.get("event") == "register", 20)
        sock = os.path.join(d, reg["endpoint"])
        cpu0 = _cpu_s(dm.proc.pid)
        r = json.loads(subprocess.run([KUBELET_STUB, "bench", "--socket", sock, "--pods", str(a.pods),
                                       "--warmup", "1000"], capture_output=True, text=True, timeout=600).stdout)
        cpu = _cpu_s(dm.proc.pid) - cpu0
        rpcs = 2 * (a.pods + 1000)  # GetPreferredAllocation + Allocate per pod, warm-up included
        print(json.dumps({"allocate_p50_us": r["allocate"]["p50_us"], "pods_per_s": r["pods_per_s"],
                          "daemon_cpu_s": round(cpu, 3), "daemon_cpu_us_per_rpc": round(cpu / rpcs * 1e6, 3)}))
    finally:
        dm.stop()
        k.stop()


if __name__ == "__main__":
    main()

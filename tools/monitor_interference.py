#!/usr/bin/env python3
"""Does the plugin's monitoring disturb the GPU's workloads? A PyTorch loop on
the GPU -- a bf16 4096^3 GEMM timed by HIP events, and a tiny kernel launched
and synchronised from the host (the path a driver lock or a busy amdsmi call
would stretch) -- runs alone, then next to the daemon on real libamd_smi with
its monitoring turned up far beyond the defaults: health polls (liveness, ECC,
retired pages, partition mode) every 50 ms, the driver-side HBM scan every
100 ms, /metrics scraped every 200 ms. Reports p50 / p99 of both timings per
phase, interleaved (off, on, off, on) so drift shows.

  python tools/monitor_interference.py [--seconds 10] [--rounds 2]

Prints one JSON object.
"""
import argparse
import json
import os
import socket
import sys
import threading
import time
import urllib.request

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_sharing_plugin_amd.utils import harness  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))], 4) if xs else None


def workload(torch, seconds):
    """(GEMM ms per call via HIP events, launch+sync us per tiny kernel)."""
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    t = torch.zeros(1, device="cuda")
    for _ in range(5):
        a @ b
    torch.cuda.synchronize()
    gemm, tiny = [], []
    t_end = time.monotonic() + seconds
    while time.monotonic() < t_end:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        a @ b
        e.record()
        e.synchronize()
        gemm.append(s.elapsed_time(e))
        for _ in range(10):
            t0 = time.perf_counter()
            t.add_(1)
            torch.cuda.synchronize()
            tiny.append((time.perf_counter() - t0) * 1e6)
    return gemm, tiny


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args(argv)
    import torch
    torch.cuda.init()
    phases = []
    for r in range(a.rounds):
        for monitored in (False, True):
            d = dm = kub = None
            stop = threading.Event()
            scrapes = [0]
            if monitored:
                d = harness.scratch_dir("adpintf")
                kub = harness.NativeKubelet(os.path.join(d, "kubelet.sock")).start()
                with socket.socket() as s0:
                    s0.bind(("127.0.0.1", 0))
                    port = s0.getsockname()[1]
                from k8s_gpu_sharing_plugin_amd import BUILD_DIR
                dm = harness.Daemon(
                    d, None, real_smi=True,
                    args=["--devices", "0", "--metrics-addr", f"127.0.0.1:{port}",
                          "--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units",
                          "--memcap-lib", os.path.join(BUILD_DIR, "libadp_memcap.so")],
                    env={"ADP_LOG_LEVEL": "warn", "DP_HEALTH_POLL_MS": "50", "DP_DRIVER_HBM_POLL_MS": "100"}).start()
                kub.wait(lambda e: e.get("event") == "devices", 30)

                def scrape():
                    while not stop.wait(0.2):
                        try:
                            with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as resp:
                                resp.read()
                            scrapes[0] += 1
                        except OSError:
                            pass
                threading.Thread(target=scrape, daemon=True).start()
                time.sleep(1)  # monitoring in full swing
            try:
                gemm, tiny = workload(torch, a.seconds)
                polls = None
                if monitored:
                    with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as resp:
                        for ln in resp.read().decode().splitlines():
                            if ln.startswith("amdgpu_dp_health_polls_total"):
                                polls = float(ln.split()[-1])
            finally:
                stop.set()
                if dm:
                    dm.stop()
                if kub:
                    kub.stop()
            phases.append({"round": r, "monitoring": monitored, "gemms": len(gemm),
                           "gemm_ms_p50": pct(gemm, 0.5), "gemm_ms_p99": pct(gemm, 0.99),
                           "tflops_p50": round(2 * 4096 ** 3 / (pct(gemm, 0.5) * 1e-3) / 1e12, 1),
                           "launch_sync_us_p50": pct(tiny, 0.5), "launch_sync_us_p99": pct(tiny, 0.99),
                           "health_polls": polls, "scrapes": scrapes[0] if monitored else None})
            print(json.dumps(phases[-1]), file=sys.stderr, flush=True)
    off = [p for p in phases if not p["monitoring"]]
    on = [p for p in phases if p["monitoring"]]
    res = {"phases": phases,
           "gemm_ms_p50_off_on": [pct([p["gemm_ms_p50"] for p in off], 0.5), pct([p["gemm_ms_p50"] for p in on], 0.5)],
           "launch_sync_us_p99_off_on": [max(p["launch_sync_us_p99"] for p in off),
                                         max(p["launch_sync_us_p99"] for p in on)]}
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

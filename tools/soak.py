"""Soak test: the daemon under continuous pod churn, periodic SIGHUP restarts,
kubelet restarts and metric scrapes; samples its RSS, open fds and threads.

  python tools/soak.py [--seconds 300] [--clients 4] [--real] [--enforce] [--holders N] [--relay]
                       [--out soak.json]

Prints one progress line per sample (every 10 s) and a final JSON summary with
pods served, restarts, and first/last/max RSS/fds/threads. Exit code 1 if the
daemon died, RSS grew by more than --max-rss-growth-mib, or fds/threads leaked.
With --relay an event relay (--event-relay) runs next to the daemon, which
takes its health events -- and, with --enforce, its driver-side scans -- from
it; the relay's RSS/fds/threads are sampled and checked the same way.
"""

import argparse
import json
import os
import signal
import subprocess
import sys
import time
import urllib.request

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_sharing_plugin_amd import KUBELET_STUB  # noqa: E402
from k8s_gpu_sharing_plugin_amd.models import fixtures  # noqa: E402
from k8s_gpu_sharing_plugin_amd.utils import harness  # noqa: E402


def proc_stats(pid):
    rss = threads = 0
    with open(f"/proc/{pid}/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                rss = int(line.split()[1]) // 1024
            elif line.startswith("Threads:"):
                threads = int(line.split()[1])
    fds = len(os.listdir(f"/proc/{pid}/fd"))
    return {"rss_mib": rss, "fds": fds, "threads": threads}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=int, default=300)
    ap.add_argument("--clients", type=int, default=4)
    ap.add_argument("--real", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--max-rss-growth-mib", type=int, default=16)
    ap.add_argument("--enforce", action="store_true",
                    help="replicas with HBM shares enforced by the HBM-cap shim (re-installed on every restart)")
    ap.add_argument("--holders", type=int, default=0,
                    help="(--real) HIP processes holding 256 MiB each during the soak: GPU processes for the "
                         "driver-side scan to find")
    ap.add_argument("--relay-restart-every", type=int, default=0,
                    help="with --relay: stop the relay every N rounds (SIGTERM and SIGKILL in turn) and start a new "
                         "one -- amdsmi registered afresh each time, the daemon reconnecting across the gap")
    ap.add_argument("--relay", action="store_true",
                    help="events and driver-side scans through an event relay process (the chart's layout)")
    ap.add_argument("--drain-churn", action="store_true",
                    help="drain and undrain GPU 0 every other round through --drain-file")
    a = ap.parse_args()
    holders = []
    if a.real and a.holders:
        code = ("import ctypes, sys\nlib = ctypes.CDLL('libamdhip64.so')\np = ctypes.c_void_p()\n"
                "rc = lib.hipMalloc(ctypes.byref(p), ctypes.c_size_t(256 << 20))\n"
                "lib.hipMemset(p, 1, ctypes.c_size_t(256 << 20)); lib.hipDeviceSynchronize()\n"
                "print('holding', rc, flush=True)\nsys.stdin.read()\n")
        for _ in range(a.holders):
            h = subprocess.Popen([sys.executable, "-c", code], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                 stderr=subprocess.DEVNULL, text=True)
            h.stdout.readline()
            holders.append(h)
    d = harness.scratch_dir("adpsoak")
    ksock = os.path.join(d, "kubelet.sock")
    kub = harness.NativeKubelet(ksock).start()
    import socket
    with socket.socket() as s0:  # a free port for the metrics endpoint
        s0.bind(("127.0.0.1", 0))
        port = s0.getsockname()[1]
    drain = os.path.join(d + ".state", "drain")
    os.makedirs(os.path.dirname(drain), exist_ok=True)
    args = ["--metrics-addr", f"127.0.0.1:{port}", "--resource-config", "gpu:gpu:4",
            "--health-state-file", os.path.join(d, "health.state"), "--drain-file", drain]
    drains = 0
    if a.real:
        args += ["--devices", "0"]
    if a.enforce:
        from k8s_gpu_sharing_plugin_amd import BUILD_DIR
        args += ["--replica-hbm-share", "--enforce-memory-units",
                 "--memcap-lib", os.path.join(BUILD_DIR, "libadp_memcap.so")]
    env = {"ADP_LOG_LEVEL": "warn", "DP_HEALTH_POLL_MS": "200"}
    if a.enforce:  # grant accounting files per pod, and the driver-side /proc scan every 100 ms
        env["DP_DRIVER_HBM_POLL_MS"] = "100"
    fx = None if a.real else dict(fixtures.node(8), events_open_kfd=True)
    relay = None
    if a.relay:
        esock = os.path.join(d + ".relay", "events.sock")
        os.makedirs(os.path.dirname(esock), exist_ok=True)
        # (info: its per-connection decisions -- registration kept or renewed -- are counted below)
        def start_relay(n):
            return harness.Daemon(d + f".relay{n}" if n else d + ".relay", fx,
                                  args=["--event-relay", "--health-event-socket", esock],
                                  real_smi=a.real, env={"ADP_LOG_LEVEL": "info"},
                                  log_path=(d + f".relay{n}.log") if n else None).start()
        relay = start_relay(0)
        deadline = time.time() + 30
        while not os.path.exists(esock):
            assert time.time() < deadline and relay.proc.poll() is None, relay.log()[-2000:]
            time.sleep(0.05)
        args += ["--health-event-socket", esock]
    dm = harness.Daemon(d, fx, args=args, real_smi=a.real, env=env).start()
    relay_samples = []
    driver_polls = None
    scans = []  # (source, processes, descriptors, seconds) of the last scan, per scrape
    samples, pods, hups, kubelet_restarts, scrapes = [], 0, 0, 0, 0
    daemon_counts = {}  # the daemon's own relay counters, last scrape
    relay_restarts, relay_logs = 0, []
    ok = True
    t_end = time.time() + a.seconds
    next_sample = time.time()
    try:
        reg = kub.wait(lambda e: e.get("event") == "register", 30)
        sock = os.path.join(d, reg["endpoint"])
        round_no = 0
        while time.time() < t_end:
            round_no += 1
            procs = [subprocess.Popen([KUBELET_STUB, "bench", "--socket", sock, "--pods", "3000", "--warmup", "0",
                                       "--rank", str(r), "--world", str(a.clients)],
                                      stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
                     for r in range(a.clients)]
            for p in procs:
                out, _ = p.communicate(timeout=120)
                if p.returncode == 0 and out.strip():
                    pods += json.loads(out)["pods"]
            if dm.proc.poll() is not None:
                ok = False
                print("daemon died", flush=True)
                break
            if a.drain_churn:  # GPU 0 in and out of service (by node index)
                if round_no % 2:
                    with open(drain, "w") as f:
                        f.write("0\n")
                    drains += 1
                elif os.path.exists(drain):
                    os.unlink(drain)
            # every 5th round: SIGHUP (full restart); every 7th: kubelet restart
            if round_no % 5 == 0:
                mark = len(kub.events)
                dm.signal(signal.SIGHUP)
                hups += 1
                reg = kub.wait(lambda e: e.get("event") == "register", 30, since=mark)
            if relay and a.relay_restart_every and round_no % a.relay_restart_every == 0:
                if relay_restarts % 2:
                    relay.proc.kill()
                    relay.proc.wait(timeout=30)
                else:
                    relay.stop()
                relay_logs.append(relay.log())  # after it stopped: every line it wrote
                relay_restarts += 1
                os.makedirs(d + f".relay{relay_restarts}", exist_ok=True)
                relay = start_relay(relay_restarts)
                relay_samples = []  # a new process: its own baseline
            if round_no % 7 == 0:
                kub.stop()
                kub = harness.NativeKubelet(ksock).start()
                kubelet_restarts += 1
                reg = kub.wait(lambda e: e.get("event") == "register", 30)
            sock = os.path.join(d, reg["endpoint"])
            with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
                scan = {}
                for line in r.read().decode().splitlines():
                    if line.startswith("amdgpu_dp_driver_hbm_polls_total "):
                        driver_polls = int(line.split()[1])
                    elif line.startswith("amdgpu_dp_driver_hbm_scan_processes{"):
                        scan["source"] = line.split('source="')[1].split('"')[0]
                        scan["processes"] = int(line.split()[-1])
                    elif line.startswith("amdgpu_dp_driver_hbm_scan_descriptors "):
                        scan["descriptors"] = int(line.split()[-1])
                    elif line.startswith("amdgpu_dp_driver_hbm_scan_seconds "):
                        scan["ms"] = float(line.split()[-1]) * 1e3
                    elif line.startswith(("amdgpu_dp_event_relay_disconnects_total ",
                                          "amdgpu_dp_health_event_gaps_total ")):
                        daemon_counts[line.split()[0]] = int(float(line.split()[1]))
                if scan.get("ms"):
                    scans.append(scan)
            scrapes += 1
            if time.time() >= next_sample:
                s = proc_stats(dm.proc.pid)
                s.update({"t": round(a.seconds - (t_end - time.time()), 1), "pods": pods})
                samples.append(s)
                if relay:
                    r_ = proc_stats(relay.proc.pid)
                    relay_samples.append(r_)
                    s = dict(s, relay=r_)
                print(json.dumps(s), flush=True)
                next_sample = time.time() + 10
            if relay and relay.proc.poll() is not None:
                ok = False
                print("relay died", flush=True)
                break
    finally:
        code = dm.stop()
        kub.stop()
        relay_code = relay.stop() if relay and relay.proc.poll() is None else (relay.proc.returncode if relay else None)
        for h in holders:
            h.stdin.close()
            h.wait(timeout=30)
    if code not in (0, None):
        ok = False
    warm = samples[min(2, len(samples) - 1)] if samples else {}
    last = samples[-1] if samples else {}
    summary = {
        "seconds": a.seconds, "clients": a.clients, "real_amdsmi": a.real, "enforce": a.enforce, "pods": pods,
        "sighups": hups,
        "kubelet_restarts": kubelet_restarts, "metric_scrapes": scrapes, "samples": len(samples),
        "rss_mib_after_warmup": warm.get("rss_mib"), "rss_mib_last": last.get("rss_mib"),
        "rss_mib_max": max((s["rss_mib"] for s in samples), default=None),
        "fds_after_warmup": warm.get("fds"), "fds_last": last.get("fds"),
        "threads_after_warmup": warm.get("threads"), "threads_last": last.get("threads"),
        "exit_code": code, "driver_hbm_polls": driver_polls, "holders": len(holders), "drains": drains,
    }
    if scans:
        ms = sorted(s["ms"] for s in scans)
        summary["driver_scan"] = {
            "scrapes": len(scans), "sources": sorted({s.get("source", "?") for s in scans}),
            "processes_max": max(s.get("processes", 0) for s in scans),
            "descriptors_max": max(s.get("descriptors", 0) for s in scans),
            "ms_p50": round(ms[len(ms) // 2], 3), "ms_max": round(ms[-1], 3)}
    if samples and last["rss_mib"] - warm["rss_mib"] > a.max_rss_growth_mib:
        ok = False
    if samples and (last["fds"] > warm["fds"] + 4 or last["threads"] > warm["threads"] + 2):
        ok = False
    if relay:
        rw = relay_samples[min(2, len(relay_samples) - 1)] if relay_samples else {}
        rl = relay_samples[-1] if relay_samples else {}
        rlog = "".join(relay_logs) + relay.log()
        summary["relay"] = {"exit_code": relay_code, "rss_mib_after_warmup": rw.get("rss_mib"),
                            "restarts": relay_restarts,
                            "relays": relay_restarts + 1,
                            "registrations": rlog.count("event notification registered on"),
                            "registration_failures": (rlog.count("event notification unavailable")
                                                      + rlog.count("events=off reason")),
                            "daemon_connections": rlog.count("daemon connected for events"),
                            "registration_kept": rlog.count("registration kept"),
                            "registration_renewed": rlog.count("re-enumerating"),
                            "nothing_missed": rlog.count("nothing missed"),
                            # the daemon's side: connections lost (one per relay restart, plus
                            # any drop) and event gaps it recorded
                            "daemon_relay_disconnects": daemon_counts.get(
                                "amdgpu_dp_event_relay_disconnects_total"),
                            "daemon_event_gaps": daemon_counts.get("amdgpu_dp_health_event_gaps_total"),
                            "rss_mib_last": rl.get("rss_mib"), "fds_after_warmup": rw.get("fds"),
                            "fds_last": rl.get("fds"), "threads_after_warmup": rw.get("threads"),
                            "threads_last": rl.get("threads")}
        if relay_code not in (0, None) or summary["relay"]["registration_failures"]:
            ok = False
        if relay_samples and (rl["rss_mib"] - rw["rss_mib"] > a.max_rss_growth_mib or rl["fds"] > rw["fds"] + 4
                              or rl["threads"] > rw["threads"] + 2):
            ok = False
    summary["ok"] = ok
    print(json.dumps(summary), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"summary": summary, "samples": samples}, f, indent=1)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())

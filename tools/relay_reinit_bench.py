"""The event relay's registration renewals on the amdsmi in use: real
libamd_smi on a GPU box, the mock here (--mock).

    python tools/relay_reinit_bench.py [--mock] [--rounds N] [--out FILE]

Measures, one JSON document:
  connect      connect -> first hello (ms)
  renew        a bare "reinit" (an older daemon: amdsmi shut_down + init,
               re-enumerate, register events again) -> its reinit hello: the
               client's round trip and the relay's own renew_ms
  kept         "reinit fp=<the registration's fingerprint>" -> its reinit hello
               (nothing re-enumerated)
  scan_during_renew
               driver-side scans issued while renewals run: their latency (the
               relay's poll loop no longer waits for a renewal)
  restarts     fresh relay processes: did event registration succeed each time
               (real amdsmi: /dev/kfd, the KFD event queue)
  daemon       the plugin daemon against the relay, plain and under the device-
               cgroup simulator (an unprivileged pod): does its view of the
               processors match the relay's, so its SIGHUPs keep the
               registration ("registration kept") instead of renewing it
"""
import argparse
import json
import os
import signal
import socket
import statistics
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_sharing_plugin_amd import BUILD_DIR  # noqa: E402
from k8s_gpu_sharing_plugin_amd.models import fixtures  # noqa: E402
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet  # noqa: E402

SIM = os.path.join(BUILD_DIR, "libadp_devcgroup_sim.so")


def kv(line, key):
    for tok in line.split(" reason=")[0].split():
        if tok.startswith(key + "="):
            return tok[len(key) + 1:]
    return None


class Conn:
    def __init__(self, path, timeout=30):
        self.s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.s.settimeout(timeout)
        t0 = time.perf_counter()
        self.s.connect(path)
        self.buf = b""
        self.hello = self.line()
        self.connect_ms = (time.perf_counter() - t0) * 1e3

    def line(self):
        while b"\n" not in self.buf:
            chunk = self.s.recv(65536)
            if not chunk:
                raise EOFError("relay closed the connection")
            self.buf += chunk
        ln, self.buf = self.buf.split(b"\n", 1)
        return ln.decode()

    def reinit(self, req):
        t0 = time.perf_counter()
        self.s.sendall((req + "\n").encode())
        while True:
            ln = self.line()
            if ln.startswith("hello v1 reinit "):
                return (time.perf_counter() - t0) * 1e3, ln

    def close(self):
        self.s.close()


def scan(path, usage):
    t0 = time.perf_counter()
    c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    c.settimeout(30)
    c.connect(path)
    c.sendall(f"scan\t{usage}\t0::/\n".encode())
    while c.recv(65536):
        pass
    c.close()
    return (time.perf_counter() - t0) * 1e3


def pct(xs, p):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(p / 100 * len(xs)))], 3) if xs else None


def summary(xs):
    return {"n": len(xs), "p50": pct(xs, 50), "p99": pct(xs, 99), "max": round(max(xs), 3) if xs else None,
            "mean": round(statistics.mean(xs), 3) if xs else None}


def start_relay(work, fx, real, n):
    sock = os.path.join(work, "relay.sock")
    r = harness.Daemon(os.path.join(work, f"relay{n}"), fx, real_smi=real,
                       args=["--event-relay", "--health-event-socket", sock], log_path=os.path.join(work, f"relay{n}.log"))
    r.start()
    r.wait_log("relaying amdsmi events on", timeout=60)
    return r, sock


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mock", action="store_true")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--restarts", type=int, default=5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    real = not a.mock
    fx = dict(fixtures.node(2), events_open_kfd=True) if a.mock else None
    work = tempfile.mkdtemp(prefix="adp-relay-bench-")
    os.makedirs(os.path.join(work, "usage"))
    out = {"amdsmi": "real" if real else "mock", "rounds": a.rounds}
    relay, sock = start_relay(work, fx, real, 0)
    try:
        c = Conn(sock)
        out["hello"] = c.hello
        out["connect_ms"] = round(c.connect_ms, 3)
        fp = kv(c.hello, "fp")
        renew_rt, renew_ms, kept_rt = [], [], []
        for _ in range(a.rounds):
            rt, ln = c.reinit("reinit")
            renew_rt.append(rt)
            renew_ms.append(float(kv(ln, "renew_ms")))
        last = ln
        fp = kv(last, "fp")
        for _ in range(a.rounds):
            rt, ln = c.reinit(f"reinit fp={fp} since=-")
            kept_rt.append(rt)
        out["renew"] = {"round_trip_ms": summary(renew_rt), "relay_renew_ms": summary(renew_ms),
                        "last_hello": last}
        out["kept"] = {"round_trip_ms": summary(kept_rt), "last_hello": ln,
                       "renewed_anyway": relay.log().count("re-enumerating") - a.rounds}
        # scans while renewals run on the registrar thread
        scans, stop = [], threading.Event()

        def scanner():
            while not stop.is_set():
                scans.append(scan(sock, os.path.join(work, "usage")))
        th = threading.Thread(target=scanner)
        th.start()
        for _ in range(a.rounds):
            c.reinit("reinit")
        stop.set()
        th.join()
        out["scan_during_renew_ms"] = summary(scans)
        c.close()
        out["renew_log_lines"] = [ln for ln in relay.log().splitlines() if "registered on" in ln][-3:]
    finally:
        relay.stop()
    # fresh relay processes
    restarts = []
    for i in range(1, a.restarts + 1):
        t0 = time.perf_counter()
        r, sock = start_relay(work, fx, real, i)
        try:
            cc = Conn(sock)
            restarts.append({"start_to_hello_ms": round((time.perf_counter() - t0) * 1e3, 1),
                             "events": kv(cc.hello, "events"), "processors": kv(cc.hello, "processors"),
                             "renew_ms": kv(cc.hello, "renew_ms"), "reason": cc.hello.partition(" reason=")[2]})
            cc.close()
        finally:
            r.stop()
    out["restarts"] = restarts
    # the daemon against a relay: plain, and denied the device nodes
    daemons = {}
    for mode in ("plain", "devcgroup_sim"):
        r, sock = start_relay(work, fx, real, f"d-{mode}")
        pdir = os.path.join(work, f"plugins-{mode}")
        os.makedirs(pdir)
        k = kubelet.StubKubelet(os.path.join(pdir, "kubelet.sock")).start()
        env = {"DP_HEALTH_POLL_MS": "1000"}
        if mode == "devcgroup_sim":
            env["LD_PRELOAD"] = " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), SIM) if x)
        d = harness.Daemon(pdir, fx, real_smi=real, args=["--health-event-socket", sock], env=env,
                           log_path=os.path.join(work, f"daemon-{mode}.log"))
        d.start()
        try:
            d.wait_log("events on through the relay", timeout=60)
            for i in range(3):
                d.signal(signal.SIGHUP)
                d.wait_log("events on through the relay", count=i + 2, timeout=60)
            rlog = r.log()
            daemons[mode] = {"kept": rlog.count("registration kept"), "renewed": rlog.count("re-enumerating"),
                             "nothing_missed": rlog.count("nothing missed"),
                             "renew_reasons": [ln.split("re-enumerating", 1)[1] for ln in rlog.splitlines()
                                               if "re-enumerating" in ln][:2]}
        finally:
            d.stop()
            k.stop()
            r.stop()
    out["daemon"] = daemons
    text = json.dumps(out, indent=2)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()

"""Cost of the driver-side HBM scan on a busy node (memcap::ScanDriverHbm).

Builds a synthetic /proc: 8 GPU processes (a KFD fd and a render fd with DRM
fdinfo each) next to N other processes holding F descriptors each (sockets and
files), and KFD's list of the GPU processes (/sys/class/kfd/kfd/proc/<pid>).
Times the scan reading only KFD's processes against the full walk of every
process, for several N, and checks both attribute the same HBM.

  python tools/driver_scan_bench.py --others 1000,10000 --fds 100 --out profiles/r4/driver_scan/scan_cost.json

--relay also times the same scans asked of an event relay (--event-relay on the
mock, the chart's layout): connect, greeting, request, the serialized reply,
close -- what one poll of a daemon with --health-event-socket costs.
"""

import argparse
import json
import os
import shutil
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from k8s_gpu_sharing_plugin_amd.utils import native  # noqa: E402

GPU_PIDS = [4100 + i for i in range(8)]
BDF = "0000:0c:00.0"


def build(root, others, fds):
    for i, pid in enumerate(GPU_PIDS):
        base = os.path.join(root, "proc", str(pid))
        os.makedirs(os.path.join(base, "fd"))
        os.makedirs(os.path.join(base, "fdinfo"))
        os.symlink("/dev/kfd", os.path.join(base, "fd", "3"))
        os.symlink("/dev/dri/renderD128", os.path.join(base, "fd", "7"))
        kib = (1000 + i) * 1024
        with open(os.path.join(base, "fdinfo", "7"), "w") as f:
            f.write(f"pos:\t0\ndrm-driver:\tamdgpu\ndrm-client-id:\t{pid}\ndrm-pdev:\t{BDF}\n"
                    f"drm-resident-vram:\t{kib} KiB\n")
        with open(os.path.join(base, "cgroup"), "w") as f:
            f.write(f"0::/kubepods/pod{i}/ctr\n")
        with open(os.path.join(base, "maps"), "w") as f:
            f.write("")
        os.makedirs(os.path.join(root, "kfd", str(pid)))
    for n in range(others):
        fd_dir = os.path.join(root, "proc", str(100000 + n), "fd")
        os.makedirs(fd_dir)
        for fd in range(fds):
            os.symlink(f"socket:[{n * fds + fd}]" if fd % 2 else "/var/log/app.log", os.path.join(fd_dir, str(fd)))


def relay_scan(sock):
    """One scan through the relay's socket, as memcap::RemoteScan asks it: (us, reply header)."""
    import socket
    t = time.perf_counter()
    c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    c.connect(sock)
    c.sendall(b"scan\t/nonexistent/usage\t0::/bench\n")
    data = b""
    while True:
        chunk = c.recv(1 << 16)
        if not chunk:
            break
        data += chunk
    c.close()
    us = (time.perf_counter() - t) * 1e6
    header = next(ln for ln in data.decode().splitlines() if ln.startswith("scan\t")).split("\t")
    return us, {"source": header[1], "pids": int(header[2]), "fds": int(header[3]), "rows": int(header[5]),
                "reply_bytes": len(data)}


def timed_relay(proc, kfd, reps, tmp):
    from k8s_gpu_sharing_plugin_amd.models import fixtures
    from k8s_gpu_sharing_plugin_amd.utils import harness
    sock = os.path.join(tmp, "relay.sock")
    r = harness.Daemon(os.path.join(tmp, "relay"), fixtures.node(1), env={"ADP_LOG_LEVEL": "warn"}, args=[
        "--event-relay", "--health-event-socket", sock, "--host-proc", proc, "--kfd-proc-dir", kfd]).start()
    try:
        deadline = time.time() + 30
        while not os.path.exists(sock):
            assert time.time() < deadline, r.log()[-2000:]
            time.sleep(0.02)
        runs = [relay_scan(sock) for _ in range(reps)]
    finally:
        r.stop()
    return runs[-1][1], statistics.median(u for u, _ in runs)


def timed(proc, kfd, reps):
    runs = [native.driver_scan(proc, kfd_proc_dir=kfd) for _ in range(reps)]
    return runs[-1], statistics.median(r["scan_us"] for r in runs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--others", default="0,1000,10000")
    ap.add_argument("--fds", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    ap.add_argument("--relay", action="store_true", help="also time the scans through an event relay")
    a = ap.parse_args()
    rows = []
    for others in [int(x) for x in a.others.split(",")]:
        root = tempfile.mkdtemp(prefix="adpscan", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        try:
            t = time.perf_counter()
            build(root, others, a.fds)
            built_s = time.perf_counter() - t
            proc, kfd = os.path.join(root, "proc"), os.path.join(root, "kfd")
            fast, fast_us = timed(proc, kfd, a.reps)
            full, full_us = timed(proc, "", max(1, a.reps // 2))
            same = sorted((p["pid"], p["bytes"]) for p in fast["procs"]) == \
                sorted((p["pid"], p["bytes"]) for p in full["procs"])
            row = {"other_processes": others, "fds_per_other": a.fds, "gpu_processes": len(GPU_PIDS),
                   "kfd": {"pids": fast["pids_scanned"], "fds": fast["fd_entries"], "scan_us_p50": round(fast_us, 1)},
                   "full_walk": {"pids": full["pids_scanned"], "fds": full["fd_entries"],
                                 "scan_us_p50": round(full_us, 1)},
                   "same_attribution": same, "hbm_total": fast["total"], "build_s": round(built_s, 1)}
            if a.relay:
                rk, rk_us = timed_relay(proc, kfd, a.reps, root)
                rf, rf_us = timed_relay(proc, "", max(1, a.reps // 2), root)
                row["relay"] = {"kfd": dict(rk, round_trip_us_p50=round(rk_us, 1)),
                                "full_walk": dict(rf, round_trip_us_p50=round(rf_us, 1))}
            rows.append(row)
            print(json.dumps(row), flush=True)
        finally:
            shutil.rmtree(root, ignore_errors=True)
    out = {"what": "memcap::ScanDriverHbm on a synthetic /proc (tmpfs), KFD GPU-process list vs full walk"
                   + (", in process and through an event relay (round trip: connect to close)" if a.relay else ""),
           "host": os.uname().nodename, "rows": rows}
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

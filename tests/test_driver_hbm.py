"""Driver-side truth for enforced HBM grants (--driver-hbm-poll-ms).

The shim counts inside the container; the driver counts every allocation of
every process (DRM fdinfo, drm-resident-vram). The daemon reads the fdinfo of
every process under --host-proc, attributes each GPU-holding process to a grant
-- the grant's accounting file mapped in /proc/<pid>/maps, else a cgroup shared
with such a process -- and reports, per container and GPU, what the driver
counts next to the grant, whether it is over (beyond a per-process runtime
allowance) and how often it went over. CPU: a fake /proc tree with fdinfo in
the layout the MI355X box showed (profiles/r3/driver/driver_usage.json). The
real-hardware run (a ctypes hipMalloc that bypasses the shim) is
tests/test_gpu.py::test_driver_sees_an_allocation_that_bypasses_the_shim.

Reference: none -- the reference counts memory units and never looks at use
(/root/reference/cmd/nvidia-device-plugin/server.go:99-111).
"""

import os
import re
import time

import pytest

from k8s_gpu_sharing_plugin_amd import BUILD_DIR
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

from test_metrics import _get, _parse, _value

SHIM = os.path.join(BUILD_DIR, "libadp_memcap.so")
MIB = 1 << 20
BDF0 = "0000:0c:00.0"


class FakeProc:
    """<root>/<pid>/{fd/<n> -> /dev/dri/renderD*, fdinfo/<n>, maps, cgroup}."""

    def __init__(self, root):
        self.root = root
        os.makedirs(root, exist_ok=True)

    def process(self, pid, cgroup, vram_mib=None, client=None, maps_file=None, bdf=BDF0, extra_fds=(),
                maps_dev=None, maps_path="/run/amdgpu-dp/memcap", kfd=True):
        base = os.path.join(self.root, str(pid))
        os.makedirs(os.path.join(base, "fd"), exist_ok=True)
        os.makedirs(os.path.join(base, "fdinfo"), exist_ok=True)
        with open(os.path.join(base, "cgroup"), "w") as f:
            f.write(cgroup + "\n")
        maps = "55d0c0000000-55d0c0021000 r--p 00000000 08:01 131 /usr/bin/python3.10\n"
        if maps_file:
            st = os.stat(maps_file)
            dev = maps_dev or f"{os.major(st.st_dev):02x}:{os.minor(st.st_dev):02x}"
            maps += f"7f0000000000-7f0000100000 rw-s 00000000 {dev} {st.st_ino} {maps_path}\n"
        with open(os.path.join(base, "maps"), "w") as f:
            f.write(maps)
        fd = os.path.join(base, "fd", "3")
        if kfd and not os.path.lexists(fd):
            os.symlink("/dev/kfd", fd)  # the KFD fd carries no memory stats
            with open(os.path.join(base, "fdinfo", "3"), "w") as f:
                f.write("pos:\t0\n")
        if vram_mib is not None:
            self.render(pid, 7, vram_mib, client if client is not None else pid * 10, bdf)
        for n, target in extra_fds:
            p = os.path.join(base, "fd", str(n))
            if not os.path.lexists(p):
                os.symlink(target, p)

    def render(self, pid, fd, vram_mib, client, bdf=BDF0):
        base = os.path.join(self.root, str(pid))
        link = os.path.join(base, "fd", str(fd))
        if not os.path.lexists(link):
            os.symlink("/dev/dri/renderD128", link)
        kib = vram_mib * 1024
        with open(os.path.join(base, "fdinfo", str(fd)), "w") as f:
            f.write(f"pos:\t0\ndrm-driver:\tamdgpu\ndrm-client-id:\t{client}\ndrm-pdev:\t{bdf}\n"
                    f"drm-total-vram:\t{kib} KiB\ndrm-shared-vram:\t0\ndrm-resident-vram:\t{kib} KiB\n"
                    f"drm-memory-vram:\t{kib} KiB\n")


@pytest.fixture
def node(scratch, tmp_path):
    proc = FakeProc(str(tmp_path / "proc"))
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack",
        "--enforce-memory-units", "--memcap-lib", SHIM, "--host-proc", proc.root,
        "--driver-hbm-poll-ms", "50", "--driver-hbm-slack-mib", "100"]).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        resp = c.allocate(ids[:3]).container_responses[0]  # 3 units = 3000 MiB on GPU 0
        c.close()
        host = [m.host_path for m in resp.mounts if m.container_path == "/run/amdgpu-dp/memcap"][0]
        deadline = time.time() + 5
        while not os.path.isfile(host) and time.time() < deadline:
            time.sleep(0.01)
        yield d, proc, port, host
    finally:
        d.stop()
        k.stop()


def _scrape_after_poll(port, min_polls):
    deadline = time.time() + 5
    while True:
        s = _parse(_get(port, "/metrics")[1])
        if _value(s, "amdgpu_dp_driver_hbm_polls_total") >= min_polls or time.time() > deadline:
            return s
        time.sleep(0.02)


def _polls(port):
    return _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_driver_hbm_polls_total")


def test_driver_counts_attribute_every_process_of_the_container(node):
    d, proc, port, host = node
    key = os.path.basename(host).split(".")[0]
    ctr = "0::/kubepods.slice/kubepods-pod1234.slice/cri-containerd-abc.scope"
    proc.process(101, ctr, vram_mib=1000, maps_file=host)     # under the shim: maps the grant's file
    proc.process(102, ctr, vram_mib=1200)                      # same container, no shim (bypass)
    proc.process(103, "0::/kubepods.slice/other.scope", vram_mib=1024)  # another tenant, no grant
    proc.process(104, ctr, vram_mib=None)                      # a child sharing 101's DRM client
    proc.render(104, 9, 1000, client=1010)
    proc.process(105, "0::/system.slice/sshd.service")       # no GPU
    s = _scrape_after_poll(port, _polls(port) + 2)
    lab = dict(allocation=key, bdf=BDF0)
    # 1000 + 1200 (the cgroup sibling) counted once each; 104's fd is 101's client
    assert _value(s, "amdgpu_dp_container_hbm_driver_bytes", **lab) == 2200 * MIB
    assert _value(s, "amdgpu_dp_container_hbm_over_grant", **lab) == 0  # 2200 <= 3000 + 2 x 100
    assert _value(s, "amdgpu_dp_container_hbm_granted_bytes", allocation=key) == 3000 * MIB
    assert _value(s, "amdgpu_dp_gpu_hbm_driver_bytes", bdf=BDF0) == (1000 + 1200 + 1024) * MIB
    assert _value(s, "amdgpu_dp_gpu_hbm_unattributed_bytes", bdf=BDF0) == 1024 * MIB
    assert _value(s, "amdgpu_dp_driver_hbm_unreadable_processes") == 0


def test_root_cgroup_is_never_a_container(node):
    """Processes outside any container share the root cgroup: one of them
    mapping the grant's file (a host-side tool) must not pull every other host
    GPU process into the grant."""
    d, proc, port, host = node
    key = os.path.basename(host).split(".")[0]
    proc.process(301, "0::/", vram_mib=500, maps_file=host)   # maps the file itself: attributed
    proc.process(302, "0::/", vram_mib=4000)                 # another host process: not the grant's
    s = _scrape_after_poll(port, _polls(port) + 2)
    lab = dict(allocation=key, bdf=BDF0)
    assert _value(s, "amdgpu_dp_container_hbm_driver_bytes", **lab) == 500 * MIB
    assert _value(s, "amdgpu_dp_container_hbm_over_grant", **lab) == 0
    assert _value(s, "amdgpu_dp_gpu_hbm_unattributed_bytes", bdf=BDF0) == 4000 * MIB


def test_over_grant_is_flagged_and_counted_per_transition(node):
    d, proc, port, host = node
    key = os.path.basename(host).split(".")[0]
    ctr = "0::/kubepods/pod-a/ctr"
    proc.process(201, ctr, vram_mib=1000, maps_file=host)
    proc.process(202, ctr, vram_mib=2500)   # e.g. ctypes hipMalloc / HSA direct: the shim never saw it
    s = _scrape_after_poll(port, _polls(port) + 2)
    lab = dict(allocation=key, bdf=BDF0)
    assert _value(s, "amdgpu_dp_container_hbm_driver_bytes", **lab) == 3500 * MIB
    assert _value(s, "amdgpu_dp_container_hbm_over_grant", **lab) == 1    # 3500 > 3000 + 2 x 100
    assert _value(s, "amdgpu_dp_container_hbm_over_grant_total", **lab) == 1
    assert _value(s, "amdgpu_dp_hbm_over_grant_events_total") == 1
    # the shim's own count (the accounting file) saw none of it
    assert _value(s, "amdgpu_dp_container_hbm_used_bytes", allocation=key) == 0
    assert "over its grant" in d.wait_log("over its grant")
    proc.render(202, 7, 1000, client=2020)  # back under
    s = _scrape_after_poll(port, _polls(port) + 2)
    assert _value(s, "amdgpu_dp_container_hbm_over_grant", **lab) == 0
    assert _value(s, "amdgpu_dp_container_hbm_over_grant_total", **lab) == 1
    proc.render(202, 7, 2900, client=2020)  # and over again: a second transition
    s = _scrape_after_poll(port, _polls(port) + 2)
    assert _value(s, "amdgpu_dp_container_hbm_over_grant_total", **lab) == 2
    assert _value(s, "amdgpu_dp_hbm_over_grant_events_total") == 2


def test_a_forged_accounting_file_does_not_raise_the_grant(node):
    """The container can rewrite its accounting file (cap[], used[]); the granted
    bytes /metrics reports and the over-grant check uses are the daemon's own."""
    d, proc, port, host = node
    key = os.path.basename(host).split(".")[0]
    with open(host, "r+b") as f:
        f.seek(24 + 64 * 8)  # cap[0] (after the header words and used[])
        f.write((200000 * MIB).to_bytes(8, "little"))
        f.seek(24)           # used[0]
        f.write((0).to_bytes(8, "little"))
    proc.process(301, "0::/kubepods/pod-b/ctr", vram_mib=5000, maps_file=host)
    s = _scrape_after_poll(port, _polls(port) + 2)
    assert _value(s, "amdgpu_dp_container_hbm_granted_bytes", allocation=key) == 3000 * MIB
    assert _value(s, "amdgpu_dp_container_hbm_over_grant", allocation=key, bdf=BDF0) == 1


def test_attribution_through_an_overlay(node):
    """An overlay filesystem: /proc/<pid>/maps names the underlying device,
    stat() the overlay's. The same inode under the pod's mount point (or the
    grant file's own name) still identifies the grant; a same-numbered inode
    of some other file does not."""
    d, proc, port, host = node
    key = os.path.basename(host).split(".")[0]
    proc.process(501, "0::/kubepods/pod-c/a", vram_mib=700, maps_file=host, maps_dev="00:2f")
    proc.process(502, "0::/kubepods/pod-c/b", vram_mib=300, maps_file=host, maps_dev="00:30",
                 maps_path=f"/var/lib/kubelet/device-plugins/amdgpu-dp/usage/{key}.memcap")
    proc.process(503, "0::/kubepods/pod-d/c", vram_mib=400, maps_file=host, maps_dev="00:31",
                 maps_path="/usr/lib/libsomething.so")
    s = _scrape_after_poll(port, _polls(port) + 2)
    assert _value(s, "amdgpu_dp_container_hbm_driver_bytes", allocation=key, bdf=BDF0) == 1000 * MIB
    assert _value(s, "amdgpu_dp_gpu_hbm_unattributed_bytes", bdf=BDF0) == 400 * MIB


def test_unreadable_processes_are_reported(node):
    d, proc, port, host = node
    if os.geteuid() == 0:
        pytest.skip("root reads every fd directory")
    os.makedirs(os.path.join(proc.root, "401", "fd"))
    os.chmod(os.path.join(proc.root, "401", "fd"), 0)
    s = _scrape_after_poll(port, _polls(port) + 2)
    assert _value(s, "amdgpu_dp_driver_hbm_unreadable_processes") == 1


def _busy_node(root, gpu_pids, others, fds_per_other):
    """A /proc of GPU processes (render fds) and many non-GPU processes holding
    `fds_per_other` descriptors each (sockets, files): the load of a busy node."""
    proc = FakeProc(root)
    for i, pid in enumerate(gpu_pids):
        proc.process(pid, f"0::/kubepods/pod{i}/ctr", vram_mib=100 + i)
    for n in range(others):
        pid = 100000 + n
        base = os.path.join(root, str(pid))
        os.makedirs(os.path.join(base, "fd"))
        for fd in range(fds_per_other):
            os.symlink(f"socket:[{pid * 100 + fd}]" if fd % 2 else "/var/log/app.log", os.path.join(base, "fd", str(fd)))
    return proc


def _kfd_dir(path, pids):
    os.makedirs(path, exist_ok=True)
    for pid in pids:
        os.makedirs(os.path.join(path, str(pid)), exist_ok=True)  # /sys/class/kfd/kfd/proc/<pid>/
    return path


def test_scan_reads_only_the_gpu_processes_kfd_lists(tmp_path):
    """Round-3 review: the scan walked every descriptor of every process. With
    KFD's list of GPU processes (/sys/class/kfd/kfd/proc/<pid>) it reads just
    those: its work does not grow with the node's other processes, and the
    attribution is the same as the full walk's."""
    from k8s_gpu_sharing_plugin_amd.utils import native
    gpu = [4100 + i for i in range(8)]
    results = {}
    for others in (200, 2000):
        root = str(tmp_path / f"proc{others}")
        _busy_node(root, gpu, others, 50)
        kfd = _kfd_dir(str(tmp_path / f"kfd{others}"), gpu)
        fast = native.driver_scan(root, kfd_proc_dir=kfd)
        full = native.driver_scan(root)
        assert fast["pid_source"] == "kfd" and full["pid_source"] == "proc"
        assert fast["pids_scanned"] == 8 and full["pids_scanned"] == 8 + others
        assert fast["fd_entries"] == 8 * 2  # each GPU process: its KFD fd + one render fd
        assert full["fd_entries"] == 8 * 2 + others * 50
        key = lambda p: (p["pid"], p["bdf"])  # noqa: E731
        assert sorted(fast["procs"], key=key) == sorted(full["procs"], key=key)
        assert fast["total"] == full["total"] == {BDF0: sum(100 + i for i in range(8)) * MIB}
        results[others] = (fast["scan_us"], full["scan_us"])
    print("scan us (kfd, full) by non-GPU processes:", results)
    assert results[2000][1] > results[200][1]  # the full walk grows with the node


def test_kfd_pids_from_another_namespace_fall_back_to_the_full_walk(tmp_path):
    """KFD names host PIDs: with a /proc of another PID namespace none of them
    is there, so the scan walks every process rather than seeing nothing."""
    from k8s_gpu_sharing_plugin_amd.utils import native
    root = str(tmp_path / "proc")
    _busy_node(root, [41, 42], 3, 4)
    kfd = _kfd_dir(str(tmp_path / "kfd"), [900001, 900002])
    s = native.driver_scan(root, kfd_proc_dir=kfd)
    assert s["pid_source"] == "proc" and s["pids_scanned"] == 5 and len(s["procs"]) == 2
    # host PIDs that collide with unrelated processes of this /proc (no /dev/kfd
    # open there): not trusted either
    s = native.driver_scan(root, kfd_proc_dir=_kfd_dir(str(tmp_path / "kfd2"), [100000, 100001]))
    assert s["pid_source"] == "proc" and len(s["procs"]) == 2
    # no KFD directory at all (no amdgpu driver visible): the full walk too
    assert native.driver_scan(root, kfd_proc_dir=str(tmp_path / "absent"))["pid_source"] == "proc"
    # an empty KFD list is trusted: no GPU process, nothing to read
    empty = native.driver_scan(root, kfd_proc_dir=_kfd_dir(str(tmp_path / "none"), []))
    assert empty["pid_source"] == "kfd" and empty["pids_scanned"] == 0 and empty["procs"] == []


def test_render_fds_without_client_id_each_count(tmp_path):
    """Advisor round 3: a kernel whose fdinfo has no drm-client-id made every
    render fd after the first on a GPU count 0 bytes. Without an ID each
    (process, fd) counts on its own."""
    from k8s_gpu_sharing_plugin_amd.utils import native
    root = str(tmp_path / "proc")
    proc = FakeProc(root)
    for pid, mib in ((51, 300), (52, 500)):
        proc.process(pid, f"0::/kubepods/p{pid}")
        proc.render(pid, 7, mib, client=0)
        info = os.path.join(root, str(pid), "fdinfo", "7")
        text = "".join(ln for ln in open(info).read().splitlines(True) if not ln.startswith("drm-client-id"))
        open(info, "w").write(text)
    s = native.driver_scan(root)
    assert {p["pid"]: p["bytes"] for p in s["procs"]} == {51: 300 * MIB, 52: 500 * MIB}
    # with IDs, a descriptor shared by two processes still counts once
    proc.process(61, "0::/kubepods/q", vram_mib=700, client=4242)
    proc.process(62, "0::/kubepods/q", vram_mib=700, client=4242)
    s = native.driver_scan(root)
    assert sum(p["bytes"] for p in s["procs"] if p["pid"] in (61, 62)) == 700 * MIB


def test_daemon_scan_uses_the_kfd_list(scratch, tmp_path):
    proc = _busy_node(str(tmp_path / "proc"), [7001, 7002], 50, 20)
    kfd = _kfd_dir(str(tmp_path / "kfd"), [7001, 7002])
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(1), args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units",
        "--memcap-lib", SHIM, "--host-proc", proc.root, "--kfd-proc-dir", kfd, "--driver-hbm-poll-ms", "50"]).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        k.wait_registration()
        s = _scrape_after_poll(port, 2)
        assert _value(s, "amdgpu_dp_driver_hbm_scan_processes", source="kfd") == 2
        assert _value(s, "amdgpu_dp_driver_hbm_scan_descriptors") == 4
        assert _value(s, "amdgpu_dp_driver_hbm_scan_seconds") >= 0
        # the first scan walks every process (render-only holders are in no KFD list), the next ones KFD's
        assert "first scan: 52 candidate process(es) from " + proc.root in d.log()
    finally:
        d.stop()
        k.stop()


def test_scan_runs_in_the_event_relay(scratch, tmp_path):
    """With --health-event-socket the daemon asks the event relay for each scan:
    the relay (the pod's privileged container) reads the processes, the daemon
    -- here pointed at a /proc that does not exist -- needs no privilege to read
    other containers' descriptors. Over-grant detection is the same; a relay
    that goes away leaves the last scan in effect and counts the failures."""
    import signal
    proc = FakeProc(str(tmp_path / "proc"))
    kfd = _kfd_dir(str(tmp_path / "kfd"), [])
    sock = os.path.join(scratch + ".relay", "events.sock")
    os.makedirs(os.path.dirname(sock))
    fx = dict(fixtures.node(2), events_open_kfd=True)
    relay = harness.Daemon(scratch + "-relay", fx, args=[
        "--event-relay", "--health-event-socket", sock, "--host-proc", proc.root, "--kfd-proc-dir", ""]).start()
    relay.wait_log("relaying amdsmi events on")
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack",
        "--enforce-memory-units", "--memcap-lib", SHIM, "--host-proc", str(tmp_path / "nosuch"),
        "--kfd-proc-dir", kfd, "--health-event-socket", sock, "--driver-hbm-poll-ms", "50",
        "--driver-hbm-slack-mib", "100"]).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        resp = c.allocate(ids[:3]).container_responses[0]
        c.close()
        host = [m.host_path for m in resp.mounts if m.container_path == "/run/amdgpu-dp/memcap"][0]
        deadline = time.time() + 5
        while not os.path.isfile(host) and time.time() < deadline:  # written just after Allocate() answers
            time.sleep(0.01)
        key = os.path.basename(host).split(".")[0]
        ctr = "0::/kubepods/pod-r/ctr"
        proc.process(601, ctr, vram_mib=1000, maps_file=host)
        proc.process(602, ctr, vram_mib=2500)  # bypasses the shim
        s = _scrape_after_poll(port, _polls(port) + 2)
        lab = dict(allocation=key, bdf=BDF0)
        assert _value(s, "amdgpu_dp_container_hbm_driver_bytes", **lab) == 3500 * MIB
        assert _value(s, "amdgpu_dp_container_hbm_over_grant", **lab) == 1
        assert _value(s, "amdgpu_dp_driver_hbm_scan_processes", source="proc") == 2
        assert _value(s, "amdgpu_dp_driver_hbm_scan_failures_total") == 0
        assert "scans by the event relay at " + sock in d.log()
        assert "from the event relay's proc list" in d.wait_log("first scan:")
        assert "first HBM scan for a daemon" in relay.wait_log("first HBM scan for a daemon")
        # the daemon's health connection is unaffected by the scan connections
        assert "events on through the relay" in d.wait_log("events on through the relay")
        relay.signal(signal.SIGTERM)
        relay.proc.wait(timeout=10)
        d.wait_log("driver-side scan through the relay failed")
        deadline = time.time() + 5
        while _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_driver_hbm_scan_failures_total") < 2:
            assert time.time() < deadline
            time.sleep(0.05)
        s = _parse(_get(port, "/metrics")[1])
        assert _value(s, "amdgpu_dp_container_hbm_over_grant", **lab) == 1  # the last scan stays
    finally:
        d.stop()
        k.stop()
        if relay.proc.poll() is None:
            relay.stop()


def test_a_relay_that_never_answers_does_not_hold_up_shutdown(scratch, tmp_path):
    """A relay that greets and then never answers a scan: the poll waits (the
    scan is counted as failed only at its deadline), and stopping the daemon
    cancels the wait instead of sitting out the 30 s scan timeout."""
    import socket as so
    import threading
    path = os.path.join(scratch + ".mute", "events.sock")
    os.makedirs(os.path.dirname(path))
    srv = so.socket(so.AF_UNIX, so.SOCK_STREAM)
    srv.bind(path)
    srv.listen(8)
    conns = []

    def serve():
        while True:
            try:
                c, _ = srv.accept()
            except OSError:
                return
            c.sendall(b"hello v1 events=ok processors=1\n")
            conns.append(c)  # read nothing, answer nothing
    threading.Thread(target=serve, daemon=True).start()
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(1), args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units",
        "--memcap-lib", SHIM, "--health-event-socket", path, "--driver-hbm-poll-ms", "50"]).start()
    try:
        d.wait_log("scans by the event relay at")
        k.wait_registration()
        deadline = time.time() + 10
        while len(conns) < 2:  # the health monitor's connection and a scan's
            assert time.time() < deadline
            time.sleep(0.05)
        t0 = time.time()
        assert d.stop() == 0
        assert time.time() - t0 < 10
        assert "driver-side scan through the relay failed" not in d.log()
    finally:
        if d.proc.poll() is None:
            d.stop()
        k.stop()
        srv.close()
        for c in conns:
            c.close()


def test_a_malformed_relay_reply_counts_as_a_failed_scan(scratch, tmp_path):
    """A relay answering a scan with something ParseScan rejects (then closing)
    leaves the previous state and counts a failure; nothing of the reply is
    taken."""
    import socket as so
    import threading
    path = os.path.join(scratch + ".bad", "events.sock")
    os.makedirs(os.path.dirname(path))
    srv = so.socket(so.AF_UNIX, so.SOCK_STREAM)
    srv.bind(path)
    srv.listen(8)

    def serve():
        while True:
            try:
                c, _ = srv.accept()
            except OSError:
                return
            c.sendall(b"hello v1 events=ok processors=1\n")
            c.settimeout(2)
            try:
                req = c.recv(4096)
            except OSError:
                req = b""
            if req.startswith(b"scan\t"):
                c.sendall(b"scan\tproc\t1\t1\t0\t1\np\tNOTAPID\t0000:0c:00.0\t1\tk\t0\tc\n")
                c.close()
            # (the health monitor's connection stays open, silent)
    threading.Thread(target=serve, daemon=True).start()
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(1), args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units",
        "--memcap-lib", SHIM, "--health-event-socket", path, "--driver-hbm-poll-ms", "50"]).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        k.wait_registration()
        deadline = time.time() + 10
        while _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_driver_hbm_scan_failures_total") < 6:
            assert time.time() < deadline
            time.sleep(0.05)
        s = _parse(_get(port, "/metrics")[1])
        assert _value(s, "amdgpu_dp_driver_hbm_polls_total") == 0  # nothing accepted
        # judged malformed at once, not after the scan timeout
        assert "malformed scan reply" in d.wait_log("driver-side scan through the relay failed")
    finally:
        d.stop()
        k.stop()
        srv.close()


def test_a_relay_that_starts_after_the_plugin_is_waited_for(scratch, tmp_path):
    """The pod's two containers start together: polls before the relay listens
    are a wait (info), not a failure warning; the first answer says so."""
    proc = FakeProc(str(tmp_path / "proc"))
    sock = os.path.join(scratch + ".late", "events.sock")
    os.makedirs(os.path.dirname(sock))
    fx = dict(fixtures.node(1), events_open_kfd=True)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units",
        "--memcap-lib", SHIM, "--health-event-socket", sock, "--driver-hbm-poll-ms", "100"]).start()
    relay = None
    try:
        d.wait_log("driver-side scan: waiting for the event relay")
        time.sleep(0.25)  # two or three polls without a relay: inside the grace
        relay = harness.Daemon(scratch + "-relay", fx, args=[
            "--event-relay", "--health-event-socket", sock, "--host-proc", proc.root, "--kfd-proc-dir", ""]).start()
        d.wait_log("driver-side scan: the event relay answers", timeout=10)
        assert "driver-side scan through the relay failed" not in d.log()
    finally:
        d.stop()
        k.stop()
        if relay:
            relay.stop()


def test_a_render_only_holder_is_found_by_the_periodic_full_walk(scratch, tmp_path):
    """Advisor round 4: with KFD's process list the scan read only processes
    that opened /dev/kfd, so one holding HBM through a render node alone (Mesa,
    Vulkan, VA-API, a child that inherited the fd, raw amdgpu ioctls) was
    invisible -- a way around the grant. The first scan and one every
    ADP_DRIVER_FULL_WALK_MS walk every process; the render-only holders they
    find are read on every fast scan in between, so the grant's driver count
    does not flap; a new one is found within the walk period."""
    proc = FakeProc(str(tmp_path / "proc"))
    kfd_dir = str(tmp_path / "kfd")
    os.makedirs(kfd_dir)
    for pid in range(8000, 8040):  # bystanders, not GPU processes
        proc.process(pid, "0::/system.slice/x", kfd=False)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack",
        "--enforce-memory-units", "--memcap-lib", SHIM, "--host-proc", proc.root, "--kfd-proc-dir", kfd_dir,
        "--driver-hbm-poll-ms", "50", "--driver-hbm-slack-mib", "100"],
        env={"ADP_DRIVER_FULL_WALK_MS": "600"}).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        resp = c.allocate(ids[:3]).container_responses[0]  # 3000 MiB on GPU 0
        c.close()
        host = [m.host_path for m in resp.mounts if m.container_path == "/run/amdgpu-dp/memcap"][0]
        deadline = time.time() + 5
        while not os.path.isfile(host) and time.time() < deadline:
            time.sleep(0.01)
        key = os.path.basename(host).split(".")[0]
        ctr = "0::/kubepods/pod-v/ctr"
        proc.process(701, ctr, vram_mib=1000, maps_file=host)           # the HIP process, KFD lists it
        _kfd_dir(kfd_dir, [701])
        proc.process(702, ctr, vram_mib=2500, kfd=False)                # Vulkan in the same container
        lab = dict(allocation=key, bdf=BDF0)
        # fast scans see the KFD process only ...
        s = _scrape_after_poll(port, _polls(port) + 2)
        first = _value(s, "amdgpu_dp_container_hbm_driver_bytes", **lab)
        # ... until the next full walk (<= 600 ms) finds the render-only holder
        deadline = time.time() + 5
        while _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_container_hbm_driver_bytes", **lab) < 3500 * MIB:
            assert time.time() < deadline, d.log()[-2000:]
            time.sleep(0.05)
        assert first in (1000 * MIB, 3500 * MIB)
        # from then on every scan -- fast ones included -- counts it: no flapping
        bytes_seen, fast_procs = set(), set()
        polls0 = _polls(port)
        while _polls(port) < polls0 + 20:
            s = _parse(_get(port, "/metrics")[1])
            bytes_seen.add(_value(s, "amdgpu_dp_container_hbm_driver_bytes", **lab))
            fast_procs |= {v for (n, ls), v in s.items()
                           if n == "amdgpu_dp_driver_hbm_scan_processes" and dict(ls).get("source") == "kfd"}
            time.sleep(0.02)
        assert bytes_seen == {3500 * MIB}, bytes_seen
        assert fast_procs == {2}  # fast scans read KFD's process and the carried render-only one
        assert _value(s, "amdgpu_dp_container_hbm_over_grant", **lab) == 1
        assert _value(s, "amdgpu_dp_hbm_over_grant_events_total") == 1  # one transition, not one per walk
        assert _value(s, "amdgpu_dp_driver_hbm_render_only_processes") == 1
        assert "hold HBM through a render node without /dev/kfd" in d.log()
        # a second render-only holder appears: found by the next walk
        proc.process(703, ctr, vram_mib=300, kfd=False)
        deadline = time.time() + 5
        while _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_container_hbm_driver_bytes", **lab) < 3800 * MIB:
            assert time.time() < deadline
            time.sleep(0.05)
    finally:
        d.stop()
        k.stop()

"""The chart's default pod, end to end on the mock: every feature at once with
the plugin container unprivileged.

The daemon runs as the chart's drop-ALL container does: the device cgroup
denies /dev/kfd and the render nodes (libadp_devcgroup_sim.so returns EPERM;
the mock's "render_denied" makes asic_info / vram_info fail as the real
libamd_smi does then), it cannot read other processes' descriptors (its
--host-proc does not exist), and it reaches amdsmi events and the driver-side
HBM scans only through the event relay. What must still work:

* health events through the relay (a reset marks the GPU Unhealthy);
* CU-slot memory units under --replica-cu-mask (CU counts from KFD topology
  under --sysfs-root) and the packed pod's HSA_CU_MASK;
* the product label (the board's PCI product_name);
* enforced grants checked against the driver (the relay's scan sees a process
  over its grant);
* /healthz.

The real-hardware run of the same layout is
tests/test_gpu_isolation.py::test_driver_scan_through_the_relay.
"""

import os
import re
import time

from k8s_gpu_sharing_plugin_amd import BUILD_DIR
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

from test_driver_hbm import BDF0, FakeProc, MIB
from test_event_relay import SIM, _preload
from test_kfd_topology import _topology
from test_metrics import _get, _parse, _value


def test_the_default_pod_with_an_unprivileged_plugin(scratch, tmp_path):
    fx = dict(fixtures.node(2), events_open_kfd=True)
    for g in fx["gpus"]:
        g["render_denied"] = True
    sysfs = _topology(str(tmp_path / "sys"), {2: 256, 10: 256})
    for g in fx["gpus"]:
        d = os.path.join(sysfs, "bus/pci/devices", g["bdf"])
        os.makedirs(d)
        with open(os.path.join(d, "product_name"), "w") as f:
            f.write("AMD Instinct MI355 OAM\n")
    proc = FakeProc(str(tmp_path / "proc"))
    fifo = os.path.join(scratch + ".fixture", "events")
    os.makedirs(os.path.dirname(fifo))
    os.mkfifo(fifo)
    sock = os.path.join(scratch + ".fixture", "events.sock")
    relay = harness.Daemon(scratch + "-relay", fx, event_fifo=fifo, args=[
        "--event-relay", "--health-event-socket", sock, "--host-proc", proc.root, "--kfd-proc-dir", ""]).start()
    relay.wait_log("relaying amdsmi events on")
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, env={"LD_PRELOAD": _preload(SIM), "DP_HEALTH_POLL_MS": "200"}, args=[
        "--resource-config", "gpu:gpu-mem-gb:-1", "--replica-cu-mask", "--enforce-memory-units",
        "--memcap-lib", os.path.join(BUILD_DIR, "libadp_memcap.so"), "--metrics-addr", "127.0.0.1:0",
        "--health-event-socket", sock, "--host-proc", str(tmp_path / "nosuch"), "--sysfs-root", sysfs,
        "--driver-hbm-poll-ms", "50", "--driver-hbm-slack-mib", "100",
        "--node-labels-file", str(tmp_path / "labels")]).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        q, call = c.watch()
        free = [x.ID for x in q.get(timeout=5).devices]
        assert len(free) == 2 * 32  # CU-slot units, though asic_info never answered
        pod = list(c.preferred(free, size=4).container_responses[0].deviceIDs)
        r = c.allocate(pod).container_responses[0]
        envs = dict(r.envs)
        assert envs["HSA_CU_MASK"] == "0:0-31"
        unit = 294896 // 32
        assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == str(4 * unit)
        labels = dict(ln.split("=", 1) for ln in open(str(tmp_path / "labels")).read().splitlines())
        assert labels["amd.com/gpu.product"] == "AMD-Instinct-MI355-OAM"
        log = d.wait_log("events on through the relay")
        assert "device access: Operation not permitted: /dev/kfd" in log
        assert "CU counts of 2 processor(s) from KFD topology" in log
        # a process of this pod's container holding more than its 4 slots' HBM (around the shim)
        host = [m.host_path for m in r.mounts if m.container_path == "/run/amdgpu-dp/memcap"][0]
        deadline = time.time() + 5
        while not os.path.isfile(host) and time.time() < deadline:  # written just after Allocate() answers
            time.sleep(0.01)
        key = os.path.basename(host).split(".")[0]
        proc.process(701, "0::/kubepods/pod-x/ctr", vram_mib=1000, maps_file=host)
        proc.process(702, "0::/kubepods/pod-x/ctr", vram_mib=4 * unit)
        deadline = time.time() + 10
        while True:
            m = _parse(_get(port, "/metrics")[1])
            hits = [v for (n, ls), v in m.items() if n == "amdgpu_dp_container_hbm_over_grant"
                    and ("allocation", key) in ls]
            if hits == [1.0] or time.time() > deadline:
                break
            time.sleep(0.05)
        assert hits == [1.0], hits
        assert _value(m, "amdgpu_dp_container_hbm_driver_bytes", allocation=key, bdf=BDF0) == (1000 + 4 * unit) * MIB
        assert _get(port, "/healthz")[0] == 200
        # a reset event reaches the kubelet through the relay
        fd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
        os.write(fd, b"0 3 mode1 reset\n")
        os.close(fd)
        deadline = time.time() + 5
        while True:
            law = q.get(timeout=5)
            sick = sum(x.health == "Unhealthy" for x in law.devices)
            if sick == 32 or time.time() > deadline:
                break
        assert sick == 32  # every CU-slot unit of GPU 0
        call.cancel()
        c.close()
    finally:
        d.stop()
        k.stop()
        relay.stop()


def test_doctor_in_the_plugin_container(scratch, tmp_path):
    """--doctor run where the chart runs the plugin (denied device nodes, the
    relay next to it): the denial is the expected state, not a warning."""
    import subprocess
    from k8s_gpu_sharing_plugin_amd import DAEMON, MOCK_LIB
    from test_doctor import _find
    from test_event_relay import RelayNode
    n = RelayNode(scratch)
    try:
        env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, LD_PRELOAD=_preload(SIM),
                   AMDSMI_MOCK_FIXTURE=fixtures.write(n.fx, str(tmp_path / "fx")))
        r = subprocess.run([DAEMON, "--doctor", "--device-plugin-path", scratch, "--health-event-socket", n.sock],
                           capture_output=True, text=True, timeout=60, env=env)
        lines = r.stdout.splitlines()
        line = _find(lines, "device nodes:")
        assert line.startswith("ok") and "as expected for the unprivileged plugin" in line, lines
        assert _find(lines, "health events:").startswith("ok")
    finally:
        n.stop()


def _writes(log):
    try:
        lines = open(log).read().splitlines()
    except OSError:
        return []
    return [ln.split(" ", 1) for ln in lines if " " in ln]


def test_every_write_lands_on_a_mounted_volume(scratch, tmp_path):
    """readOnlyRootFilesystem: every filesystem write the plugin and the relay
    attempt (logged by libadp_devcgroup_sim.so's ADP_FS_WRITE_LOG: opens for
    writing, mkdir, rename, unlink, socket binds) falls on a volume the chart
    mounts writable -- the kubelet's plugin directory, the health-state
    hostPath (health state, drain file), the NFD features directory, the event
    socket's emptyDir, /var/run/cdi (CDI list strategies), /dev -- never on the
    container's own filesystem."""
    fx = dict(fixtures.node(2), events_open_kfd=True)
    plugin_dir = scratch  # /var/lib/kubelet/device-plugins
    state_dir = str(tmp_path / "state")  # /var/lib/amdgpu-device-plugin
    nfd_dir = str(tmp_path / "nfd")  # /etc/nfd-features
    sock_dir = scratch + ".events"  # /run/amdgpu-dp-events
    cdi_dir = str(tmp_path / "cdi")  # /var/run/cdi (mounted with a CDI list strategy)
    for d in (state_dir, nfd_dir, sock_dir, cdi_dir):
        os.makedirs(d)
    sock = os.path.join(sock_dir, "events.sock")
    dlog, rlog = str(tmp_path / "daemon.writes"), str(tmp_path / "relay.writes")
    proc = FakeProc(str(tmp_path / "proc"))
    relay = harness.Daemon(scratch + "-relay", fx, env={"LD_PRELOAD": _preload(SIM), "ADP_DEVCGROUP_ALLOW": "/dev",
                                                        "ADP_FS_WRITE_LOG": rlog}, args=[
        "--event-relay", "--health-event-socket", sock, "--host-proc", proc.root, "--kfd-proc-dir", ""]).start()
    relay.wait_log("relaying amdsmi events on")
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, env={"LD_PRELOAD": _preload(SIM), "ADP_FS_WRITE_LOG": dlog,
                                         "DP_HEALTH_POLL_MS": "100"}, args=[
        "--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units", "--memcap-lib",
        os.path.join(BUILD_DIR, "libadp_memcap.so"), "--metrics-addr", "127.0.0.1:0",
        "--health-event-socket", sock, "--host-proc", str(tmp_path / "nosuch"), "--driver-hbm-poll-ms", "50",
        "--health-state-file", os.path.join(state_dir, "health.state"),
        "--drain-file", os.path.join(state_dir, "drain"), "--node-labels-file", os.path.join(nfd_dir, "amd-gpu"),
        "--device-list-strategy", "cdi-annotations", "--cdi-spec-dir", cdi_dir])
    d.start()
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        for i in range(3):
            c.allocate(ids[i * 4:i * 4 + 4])
        c.close()
        d.wait_log("events on through the relay")
        with open(os.path.join(state_dir, "drain"), "w") as f:
            f.write(fx["gpus"][1]["bdf"] + "\n")
        d.wait_log("drained by the operator")
        os.kill(d.proc.pid, __import__("signal").SIGHUP)  # a restart re-creates sockets and files
        d.wait_log("registered device plugin", timeout=10)
    finally:
        d.stop()
        k.stop()
        relay.stop()
    allowed = [plugin_dir, state_dir, nfd_dir, sock_dir, cdi_dir, "/dev/"]
    assert any(p.startswith(cdi_dir) for _, p in _writes(dlog))  # the CDI spec was written, there
    # (a coverage build's gcov runtime writes .gcda files at exit: instrumentation, not the daemon)
    bad = {who: sorted({p for _, p in _writes(log) if not any(p.startswith(a) for a in allowed)
                        and not p.endswith(".gcda")})
           for who, log in (("daemon", dlog), ("relay", rlog))}
    assert _writes(dlog) and _writes(rlog), "the write log recorded nothing"
    assert bad == {"daemon": [], "relay": []}, bad

"""Privilege separation for health events: the event relay.

amdsmi event notification (GPU_PRE_RESET / GPU_POST_RESET) opens /dev/kfd,
which the device cgroup of an unprivileged pod denies. Instead of running the
whole plugin -- the kubelet-facing gRPC server and the /metrics HTTP server --
privileged, `amdgpu-device-plugin --event-relay` registers the events in a
second, privileged container of the same pod and forwards them over a Unix
socket (--health-event-socket); the daemon runs drop-ALL. Here the daemon runs
under libadp_devcgroup_sim.so (its /dev/kfd and render nodes answer EPERM, as
in an unprivileged pod) and the relay without it; reset events still travel.

Reference: the reference chart escalates the whole plugin (SYS_ADMIN) for MIG
monitoring, /root/reference/deployments/helm/nvidia-device-plugin/templates/daemonset.yml:80-93.
"""

import os
import re
import signal
import time

from k8s_gpu_sharing_plugin_amd import BUILD_DIR
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

from test_metrics import _get, _parse, _value

SIM = os.path.join(BUILD_DIR, "libadp_devcgroup_sim.so")


def _preload(*libs):
    return " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), *libs) if x)


class RelayNode:
    def __init__(self, scratch, relay_env=None, daemon_args=(), daemon_env=None, relay_launch=None, relay_gpus=None,
                 fx=None):
        self.scratch = scratch
        self.relay_launch = relay_launch  # argv -> argv for the relay process (e.g. another build's binary)
        self.fifo = os.path.join(scratch + ".fixture", "events")
        os.makedirs(scratch + ".fixture", exist_ok=True)
        os.mkfifo(self.fifo)
        self.sock = os.path.join(scratch + ".fixture", "events.sock")
        self.fx = dict(fx or fixtures.node(2), events_open_kfd=True)
        # The relay may see more GPUs than the daemon does (their views disagree).
        self.relay_fx = dict(fixtures.node(relay_gpus), events_open_kfd=True) if relay_gpus else self.fx
        self.relay_env = relay_env
        self.relay = None
        self.start_relay()
        self.k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        self.d = harness.Daemon(scratch, self.fx, args=["--health-event-socket", self.sock,
                                                        "--metrics-addr", "127.0.0.1:0", *daemon_args],
                                env={"LD_PRELOAD": _preload(SIM), "DP_HEALTH_POLL_MS": "200",
                                     **(daemon_env or {})}).start()
        self.port = int(re.search(r"on port (\d+)", self.d.wait_log("serving /metrics")).group(1))
        reg = self.k.wait_registration()
        self.c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        self.q, self.call = self.c.watch()
        self.first = self.q.get(timeout=5)

    def start_relay(self):
        n = 0 if self.relay is None else len(self.relay.log()) + 1
        rdir = self.scratch + f"-relay{n}"
        os.makedirs(rdir, exist_ok=True)
        self.relay = harness.Daemon(rdir, self.relay_fx, args=["--event-relay", "--health-event-socket", self.sock],
                                    env=self.relay_env, event_fifo=self.fifo, launch=self.relay_launch).start()
        self.relay.wait_log("relaying amdsmi events on")

    def inject(self, line):
        fd = os.open(self.fifo, os.O_WRONLY | os.O_NONBLOCK)
        os.write(fd, (line + "\n").encode())
        os.close(fd)

    def health(self, timeout=5):
        law = self.q.get(timeout=timeout)
        return [x.health for x in law.devices]

    def rewatch(self, timeout=15):
        """Follow the plugin's next registration (a SIGHUP restarts it); the
        first ListAndWatch of the new generation."""
        self.call.cancel()
        self.c.close()
        reg = self.k.wait_registration(timeout)
        self.c = kubelet.PluginClient(os.path.join(self.scratch, reg.endpoint))
        self.q, self.call = self.c.watch()
        return self.health()

    def wait_health(self, want, timeout=10):
        deadline = time.time() + timeout
        while True:
            h = self.health(timeout=max(0.05, deadline - time.time()))
            if h == want:
                return h

    def bdf(self, gpu):
        return self.fx["gpus"][gpu]["bdf"]

    def metrics(self):
        return _parse(_get(self.port, "/metrics")[1])

    def stop(self):
        self.call.cancel()
        self.c.close()
        self.d.stop()
        self.k.stop()
        if self.relay.proc.poll() is None:
            self.relay.stop()


def test_reset_events_travel_through_the_relay(scratch):
    n = RelayNode(scratch)
    try:
        log = n.d.wait_log("events on through the relay")
        assert "device access: Operation not permitted: /dev/kfd" in log  # the daemon itself is denied
        assert "events off:" not in log
        assert _value(n.metrics(), "amdgpu_dp_health_events_enabled") == 1
        n.inject("1 3 mode1 reset")
        assert n.health() == ["Healthy", "Unhealthy"]
        n.inject("1 4 reset done")
        assert n.health() == ["Healthy", "Healthy"]
        n.inject("0 1 page fault")  # VMFAULT: counted, health unchanged
        n.d.wait_log("VMFAULT(1) on GPU 0")
        rlog = n.relay.log()
        assert "event notification registered on 2 processor(s)" in rlog
        assert "daemon connected for events (a new daemon)" in rlog
        # The daemon's processors match the relay's registration: kept, not re-enumerated.
        assert "registration kept (a daemon's processors match it" in rlog and "re-enumerating" not in rlog
    finally:
        n.stop()


def test_daemon_reconnects_when_the_relay_restarts(scratch):
    n = RelayNode(scratch)
    try:
        n.d.wait_log("events on through the relay")
        m = n.metrics()
        assert _value(m, "amdgpu_dp_event_relay_connected") == 1
        assert _value(m, "amdgpu_dp_event_relay_disconnects_total") == 0
        first_relay = [dict(ls)["relay"] for (name, ls) in m if name == "amdgpu_dp_event_relay_info"]
        assert len(first_relay) == 1 and len(first_relay[0]) == 16, m
        n.relay.signal(signal.SIGTERM)
        n.relay.proc.wait(timeout=10)
        n.d.wait_log("event relay: the event relay closed the connection; polling only")
        m = n.metrics()
        assert _value(m, "amdgpu_dp_health_events_enabled") == 0
        assert _value(m, "amdgpu_dp_event_relay_connected") == 0
        assert _value(m, "amdgpu_dp_event_relay_disconnects_total") == 1
        n.start_relay()
        n.d.wait_log("connected to the event relay", timeout=10)
        deadline = time.time() + 10
        while _value(n.metrics(), "amdgpu_dp_health_events_enabled") != 1:
            assert time.time() < deadline
            time.sleep(0.1)
        n.inject("0 3 reset")
        assert n.health() == ["Unhealthy", "Healthy"]
        import subprocess
        import sys
        st = subprocess.run([sys.executable, "-m", "k8s_gpu_sharing_plugin_amd", "status",
                             f"http://127.0.0.1:{n.port}/metrics"], capture_output=True, text=True, timeout=60)
        assert "event relay connected (1 connection(s) lost)" in st.stdout, st.stdout
        m = n.metrics()
        relays = [dict(ls)["relay"] for (name, ls) in m if name == "amdgpu_dp_event_relay_info"]
        assert len(relays) == 1 and relays != first_relay  # a new relay instance
        assert _value(m, "amdgpu_dp_event_relay_last_event_seq") == 1
    finally:
        n.stop()


def test_relay_without_kfd_reports_events_off(scratch):
    """A relay that is itself denied /dev/kfd (not privileged) says so to the
    daemon, which polls and names the relay's reason."""
    n = RelayNode(scratch, relay_env={"LD_PRELOAD": _preload(SIM)})
    try:
        log = n.d.wait_log("event relay reports")
        line = [ln for ln in log.splitlines() if "event relay reports" in ln][0]
        assert "relay: " in line and "/dev/kfd not openable (EPERM) in the relay's container" in line
        assert _value(n.metrics(), "amdgpu_dp_health_events_enabled") == 0
        assert n.first.devices and all(x.health == "Healthy" for x in n.first.devices)
    finally:
        n.stop()


def test_daemon_serves_while_the_relay_is_absent(scratch):
    """No relay yet: devices are served, health is polled, and the daemon keeps
    trying the socket."""
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(1), args=["--health-event-socket", scratch + ".nosuch.sock"],
                       env={"DP_HEALTH_POLL_MS": "100"}).start()
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        assert [x.health for x in c.watch()[0].get(timeout=5).devices] == ["Healthy"]
        log = d.wait_log("health poll #1")
        assert "events via relay" in log and "not reachable" in log
        c.close()
    finally:
        d.stop()
        k.stop()


def test_relay_refuses_without_a_socket(scratch):
    import subprocess
    r = subprocess.run([harness.DAEMON, "--device-plugin-path", scratch, "--event-relay"], capture_output=True,
                       text=True, timeout=30, env=harness.Daemon(scratch, fixtures.node(1)).env)
    assert r.returncode == 1 and "--event-relay needs --health-event-socket" in r.stdout + r.stderr


def test_doctor_asks_the_relay(scratch, tmp_path):
    """--doctor with --health-event-socket: the relay's hello is the verdict
    (the daemon's own container is not expected to open /dev/kfd)."""
    import subprocess
    from test_doctor import _doctor, _find
    n = RelayNode(scratch)
    try:
        _, lines = _doctor(tmp_path, "--device-plugin-path", scratch, "--health-event-socket", n.sock, fx=n.fx)
        line = _find(lines, "health events:")
        assert line.startswith("ok") and "through the event relay" in line and "events=ok processors=2" in line
        # enforced grants: the driver-side scan is the relay's too
        enforced = ("--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units", "--metrics-addr",
                    "127.0.0.1:0", "--memcap-lib", os.path.join(BUILD_DIR, "libadp_memcap.so"))
        _, lines = _doctor(tmp_path, "--device-plugin-path", scratch, "--health-event-socket", n.sock, *enforced,
                           fx=n.fx)
        line = _find(lines, "driver-side HBM check")
        assert line.startswith("ok") and "the event relay reads" in line, lines
    finally:
        n.stop()
    _, lines = _doctor(tmp_path, "--device-plugin-path", scratch, "--health-event-socket", n.sock + ".gone")
    line = _find(lines, "health events:")
    assert line.startswith("warn") and "not reachable" in line
    _, lines = _doctor(tmp_path, "--device-plugin-path", scratch, "--health-event-socket", n.sock + ".gone", *enforced)
    line = _find(lines, "driver-side HBM check")
    assert line.startswith("warn") and "ran no scan" in line and "--event-relay" in line, lines


def test_relay_answers_scan_requests_and_drops_malformed_ones(scratch, tmp_path):
    """The relay's second request: one driver-side scan per connection, the
    reply in SerializeScan's lines, then the connection closes. A request whose
    directory is relative or climbs out ("..") is dropped unanswered."""
    import socket as so
    sock = str(tmp_path / "events.sock")
    fx = dict(fixtures.node(1), events_open_kfd=True)
    relay = harness.Daemon(scratch + "-relay", fx, args=["--event-relay", "--health-event-socket", sock,
                                                         "--host-proc", str(tmp_path / "proc")]).start()
    os.makedirs(str(tmp_path / "proc"))

    def ask(line):
        c = so.socket(so.AF_UNIX, so.SOCK_STREAM)
        c.settimeout(10)
        c.connect(sock)
        c.sendall(line.encode())
        data = b""
        while True:
            chunk = c.recv(65536)
            if not chunk:
                break
            data += chunk
        c.close()
        return data.decode()
    try:
        relay.wait_log("relaying amdsmi events on")
        out = ask(f"scan\t{tmp_path}/usage\t0::/\n")
        lines = out.splitlines()
        assert lines[0].startswith("hello v1 ") and lines[1].split("\t")[:2] == ["scan", "proc"], out
        assert lines[1].split("\t")[-1] == "0" and len(lines) == 2  # an empty /proc: no process rows
        for bad in ("scan\trelative/dir\tx\n", f"scan\t{tmp_path}/../etc\tx\n", "scan\tnotab\n"):
            out = ask(bad)
            assert "scan\t" not in out, (bad, out)
        assert relay.log().count("malformed scan request dropped") == 3
        # an empty /proc (the relay's own PID namespace, not the host's): said once
        assert relay.log().count("is the host's /proc mounted there (--host-proc)?") == 1
    finally:
        relay.stop()


def test_a_stuck_event_wait_turns_events_off_until_it_returns(scratch):
    """Watchdog: an amdsmi event wait that does not return (the mock's "hang")
    for ADP_RELAY_STUCK_MS is reported to the daemon as events off -- it polls
    -- and, once the wait returns, as events on again; events then flow."""
    n = RelayNode(scratch, relay_env={"ADP_RELAY_STUCK_MS": "300"})
    try:
        n.d.wait_log("events on through the relay")
        n.inject("hang 1500")
        log = n.d.wait_log("has not returned for")
        line = [ln for ln in log.splitlines() if "has not returned for" in ln][0]
        assert "event relay reports" in line and "polling only" in line, line
        deadline = time.time() + 5
        while _value(n.metrics(), "amdgpu_dp_health_events_enabled") != 0:
            assert time.time() < deadline
            time.sleep(0.05)
        assert "daemons fall back to polling" in n.relay.wait_log("daemons fall back to polling")
        n.relay.wait_log("the amdsmi event wait returned again", timeout=10)
        deadline = time.time() + 5
        while _value(n.metrics(), "amdgpu_dp_health_events_enabled") != 1:
            assert time.time() < deadline
            time.sleep(0.05)
        n.inject("1 3 mode1 reset")
        assert n.health() == ["Healthy", "Unhealthy"]
    finally:
        n.stop()


def test_relay_ping_is_the_relays_liveness(scratch, tmp_path):
    """--relay-ping (the relay container's exec liveness probe): 0 for a relay
    that greets -- events off for a lasting reason included, a restart would
    not fix that -- 1 for no relay, a relay that never greets, and a relay
    whose amdsmi event wait is stuck."""
    import socket as so
    import subprocess

    def ping(sock):
        r = subprocess.run([harness.DAEMON, "--relay-ping", "--health-event-socket", sock], capture_output=True,
                           text=True, timeout=30)
        return r.returncode, r.stdout
    assert ping(str(tmp_path / "none.sock"))[0] == 1
    mute = so.socket(so.AF_UNIX, so.SOCK_STREAM)
    mute.bind(str(tmp_path / "mute.sock"))
    mute.listen(1)
    try:
        rc, out = ping(str(tmp_path / "mute.sock"))
        assert rc == 1 and "did not greet" in out
    finally:
        mute.close()
    n = RelayNode(scratch, relay_env={"ADP_RELAY_STUCK_MS": "300"})
    try:
        rc, out = ping(n.sock)
        assert rc == 0 and out.startswith("hello v1 events=ok"), out
        n.inject("hang 2000")
        n.relay.wait_log("daemons fall back to polling")
        rc, out = ping(n.sock)
        assert rc == 1 and "has not returned" in out, out
    finally:
        n.stop()
    os.makedirs(scratch + "b")
    denied = RelayNode(scratch + "b", relay_env={"LD_PRELOAD": _preload(SIM)})
    try:
        rc, out = ping(denied.sock)
        assert rc == 0 and "events=off" in out, out
    finally:
        denied.stop()


def test_a_failing_event_wait_turns_events_off_too(scratch):
    """An event wait that keeps failing (after a GPU reset amdsmi may answer
    every wait with an error) delivers no events either: after
    ADP_RELAY_STUCK_MS of failures the daemon is told events are off, the relay
    ping fails (a restart re-initialises amdsmi), and a daemon's reinit is
    still served; once the waits succeed, events are on again."""
    import subprocess
    n = RelayNode(scratch, relay_env={"ADP_RELAY_STUCK_MS": "500"})
    try:
        n.d.wait_log("events on through the relay")
        n.inject("fail 30")  # ~3 s of failed waits (the relay retries every 100 ms)
        n.relay.wait_log("the amdsmi event wait has failed for")
        deadline = time.time() + 5
        while _value(n.metrics(), "amdgpu_dp_health_events_enabled") != 0:
            assert time.time() < deadline
            time.sleep(0.05)
        r = subprocess.run([harness.DAEMON, "--relay-ping", "--health-event-socket", n.sock], capture_output=True,
                           text=True, timeout=30)
        assert r.returncode == 1 and "has failed for" in r.stdout, r.stdout
        n.relay.wait_log("the amdsmi event wait returned again", timeout=10)
        deadline = time.time() + 5
        while _value(n.metrics(), "amdgpu_dp_health_events_enabled") != 1:
            assert time.time() < deadline
            time.sleep(0.05)
        assert "event wait failed (1 in a row)" in n.relay.log()
    finally:
        n.stop()


def test_relay_keeps_no_descriptor_per_scan(scratch, tmp_path):
    """Hundreds of scan connections (one per daemon poll in production), some
    dropped before the reply: the relay's open descriptors and threads do not
    grow."""
    import socket as so
    sock = str(tmp_path / "events.sock")
    fx = dict(fixtures.node(1), events_open_kfd=True)
    os.makedirs(str(tmp_path / "proc"))
    relay = harness.Daemon(scratch + "-relay", fx, args=["--event-relay", "--health-event-socket", sock,
                                                         "--host-proc", str(tmp_path / "proc")]).start()

    def counts():
        pid = relay.proc.pid
        threads = int([ln for ln in open(f"/proc/{pid}/status") if ln.startswith("Threads:")][0].split()[1])
        return len(os.listdir(f"/proc/{pid}/fd")), threads

    def scan(read_reply):
        c = so.socket(so.AF_UNIX, so.SOCK_STREAM)
        c.settimeout(10)
        c.connect(sock)
        c.sendall(f"scan\t{tmp_path}/usage\t0::/x\n".encode())
        if read_reply:
            while c.recv(65536):
                pass
        c.close()
    try:
        relay.wait_log("relaying amdsmi events on")
        # the registrar registers and starts the event waiter after that line:
        # count once all four threads (loop, registrar, waiter, scan worker) run
        relay.wait_log("event notification registered on")
        deadline = time.time() + 5
        while counts()[1] < 4 and time.time() < deadline:
            time.sleep(0.02)
        scan(True)
        before = counts()
        for i in range(400):
            scan(i % 4 != 0)  # every 4th client hangs up without reading
        time.sleep(0.3)
        after = counts()
        assert after[0] <= before[0] + 2 and after[1] == before[1], (before, after)
    finally:
        relay.stop()


def test_partition_events_through_the_relay(scratch):
    """CPX: each compute partition is its own amdsmi processor and KFD node.
    A reset event of one partition, relayed by KFD node, marks its GPU -- all
    of that GPU's partitions (a reset is device-wide), partitionStrategy single
    -- Unhealthy, and none of the other GPU's."""
    fifo = os.path.join(scratch + ".fixture", "events")
    os.makedirs(os.path.dirname(fifo))
    os.mkfifo(fifo)
    sock = os.path.join(scratch + ".fixture", "events.sock")
    fx = dict(fixtures.node(2, ["CPX", "CPX"], memory="NPS2"), events_open_kfd=True)
    relay = harness.Daemon(scratch + "-relay", fx, args=["--event-relay", "--health-event-socket", sock],
                           event_fifo=fifo).start()
    relay.wait_log("relaying amdsmi events on")
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, args=["--partition-strategy", "single", "--health-event-socket", sock],
                       env={"LD_PRELOAD": _preload(SIM)}).start()
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        q, call = c.watch()
        first = q.get(timeout=5)
        assert len(first.devices) == 16
        d.wait_log("events on through the relay")
        assert "event notification registered on 16 processor(s)" in relay.log()
        fd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
        os.write(fd, b"1:3 3 partition reset\n")
        os.close(fd)
        law = q.get(timeout=5)
        bdf1 = fx["gpus"][1]["bdf"][:-1]  # partitions report their own function numbers
        sick = sorted(x.ID for x in law.devices if x.health == "Unhealthy")
        assert len(sick) == 8, [x.health for x in law.devices]
        assert " node=13 " in relay.log()  # KFD node 2 + 8*1 + partition 3
        d.wait_log("GPU_PRE_RESET")
        assert bdf1 in d.log()
        call.cancel()
        c.close()
    finally:
        d.stop()
        k.stop()
        relay.stop()


def test_relay_refuses_other_uids(scratch, tmp_path):
    """The socket is its owner's only; behind that the relay checks the peer's
    credentials (SO_PEERCRED) and closes connections from another uid, even if
    the socket file was made world-writable."""
    import subprocess
    import sys
    if os.geteuid() != 0:
        import pytest
        pytest.skip("needs root to connect as another uid")
    import shutil
    import tempfile
    sdir = tempfile.mkdtemp(prefix="adp-uid-", dir="/tmp")  # traversable by another uid
    os.chmod(sdir, 0o755)
    sock = os.path.join(sdir, "events.sock")
    fx = dict(fixtures.node(1), events_open_kfd=True)
    relay = harness.Daemon(scratch + "-relay", fx, args=["--event-relay", "--health-event-socket", sock]).start()
    try:
        relay.wait_log("relaying amdsmi events on")
        assert os.stat(sock).st_mode & 0o077 == 0  # owner only
        os.chmod(sock, 0o666)
        code = ("import socket, sys\n"
                "c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM); c.settimeout(5); c.connect(sys.argv[1])\n"
                "print(repr(c.recv(100)))\n")
        r = subprocess.run([sys.executable, "-c", code, sock], capture_output=True, text=True, timeout=30,
                           preexec_fn=lambda: os.setuid(65534))
        assert r.stdout.strip() == "b''", r.stdout + r.stderr  # closed without a greeting
        assert "connection from uid 65534 refused" in relay.wait_log("refused")
    finally:
        relay.stop()
        shutil.rmtree(sdir, ignore_errors=True)


# --- event gaps: a GPU_POST_RESET nobody received ----------------------------------


def _series(metrics, name, bdf):
    for (n, labels), v in metrics.items():
        if n == name and dict(labels).get("bdf") == bdf:
            return v
    return None


def test_relay_killed_between_pre_and_post_reset_recovers_by_polling(scratch):
    """GPU_PRE_RESET arrives, then the relay dies (SIGKILL) and the reset
    completes while nobody is registered: the GPU_POST_RESET is lost. The new
    relay cannot replay it (another relay instance), so the daemon records an
    event gap on the waiting GPU; once amdsmi has answered every poll for
    --reset-recovery-hold-ms it is Healthy again, logged and counted. The other
    GPU never changes."""
    n = RelayNode(scratch, daemon_args=["--reset-recovery-hold-ms", "2500"])
    try:
        n.d.wait_log("events on through the relay")
        n.inject("1 3 mode1 reset")
        assert n.health() == ["Healthy", "Unhealthy"]
        t_kill = time.time()
        n.relay.proc.kill()
        n.relay.proc.wait(timeout=10)
        n.d.wait_log("event relay: the event relay closed the connection")
        n.start_relay()  # (the reset's POST happened in between: nobody received it)
        n.d.wait_log("renewed its registration or no longer holds the events missed", timeout=10)
        log = n.d.wait_log("waits for GPU_POST_RESET across an event gap")
        assert n.bdf(1) in log
        m = n.metrics()
        assert _series(m, "amdgpu_dp_gpu_awaiting_polled_recovery", n.bdf(1)) == 1
        assert _series(m, "amdgpu_dp_gpu_awaiting_polled_recovery", n.bdf(0)) == 0
        assert n.wait_health(["Healthy", "Healthy"], timeout=15) == ["Healthy", "Healthy"]
        assert time.time() - t_kill >= 2.4  # not before the hold
        line = [ln for ln in n.d.log().splitlines() if "recovered without GPU_POST_RESET" in ln]
        assert len(line) == 1 and n.bdf(1) in line[0] and "amdsmi answered every poll for" in line[0], line
        m = n.metrics()
        assert _series(m, "amdgpu_dp_gpu_recovered_without_event_total", n.bdf(1)) == 1
        assert _series(m, "amdgpu_dp_gpu_recovered_without_event_total", n.bdf(0)) == 0
        assert _series(m, "amdgpu_dp_gpu_awaiting_polled_recovery", n.bdf(1)) == 0
        assert _value(m, "amdgpu_dp_health_event_gaps_total") >= 1
        # events flow through the new relay as before
        n.inject("0 3 reset")
        assert n.health() == ["Unhealthy", "Healthy"]
    finally:
        n.stop()


def test_events_missed_across_a_sighup_are_replayed(scratch):
    """The daemon's SIGHUP closes its relay connection for a moment (a new
    monitor generation); a GPU_POST_RESET relayed meanwhile is replayed to the
    new connection, so the GPU is Healthy at once -- not after the polled
    hold, which is set out of reach here -- and the relay kept its registration
    (the daemon's processors match it)."""
    n = RelayNode(scratch, daemon_args=["--reset-recovery-hold-ms", "600000"],
                  daemon_env={"ADP_DEBUG_PUBLISH_DELAY_MS": "800"})
    try:
        n.d.wait_log("events on through the relay")
        n.inject("1 3 mode1 reset")
        assert n.health() == ["Healthy", "Unhealthy"]
        n.d.signal(signal.SIGHUP)
        n.d.wait_log("retrieving plugins", count=2)  # the old monitor is stopped: nobody subscribed
        n.inject("1 4 reset done")
        n.relay.wait_log(" type=4 ")  # relayed while the daemon was away
        first = n.rewatch()
        if first != ["Healthy", "Healthy"]:
            n.wait_health(["Healthy", "Healthy"], timeout=5)
        rlog = n.relay.wait_log("replaying 1 event(s)")
        assert "daemon connected for events (nothing missed)" in rlog
        assert "re-enumerating" not in rlog and rlog.count("registration kept") == 2
        assert "recovered without GPU_POST_RESET" not in n.d.log()
        assert "across an event gap" not in n.d.log()
    finally:
        n.stop()


def test_a_pre_reset_without_a_gap_keeps_waiting(scratch):
    """No gap since GPU_PRE_RESET (SIGHUPs only: the relay replays what the
    daemon missed and says nothing was lost): the GPU waits for its
    GPU_POST_RESET however long amdsmi answers -- today's rule -- and the event
    still ends the wait."""
    n = RelayNode(scratch, daemon_args=["--reset-recovery-hold-ms", "500"])
    try:
        n.d.wait_log("events on through the relay")
        n.inject("0 3 pre-reset")
        assert n.health() == ["Unhealthy", "Healthy"]
        for i in range(2):
            n.d.signal(signal.SIGHUP)
            assert n.rewatch() == ["Unhealthy", "Healthy"]
        n.relay.wait_log("daemon connected for events (nothing missed)", count=2)
        time.sleep(2.0)  # four times the hold, ten polls
        assert "recovered without GPU_POST_RESET" not in n.d.log()
        assert n.q.empty() or all(h[0] == "Unhealthy" for h in [n.health(0.1)])
        n.inject("0 4 post-reset")
        n.wait_health(["Healthy", "Healthy"])
    finally:
        n.stop()


def test_sighup_storm_with_interleaved_resets_leaves_no_gpu_stuck(scratch):
    """SIGHUPs back to back with GPU_PRE_RESET / GPU_POST_RESET pairs injected
    at every point of the restart -- before, during and after the daemon's
    reconnection -- and one relay restart in the middle: every GPU ends
    Healthy, by the events themselves (the polled hold is out of reach), and
    the relay never re-enumerated for a daemon whose processors it had."""
    import random
    rnd = random.Random(5)
    n = RelayNode(scratch, daemon_args=["--reset-recovery-hold-ms", "600000", "--reset-flap-limit", "0"])
    try:
        n.d.wait_log("events on through the relay")
        for i in range(16):
            gpu = i % 2
            n.inject(f"{gpu} 3 storm pre {i}")
            n.d.signal(signal.SIGHUP)
            time.sleep(rnd.uniform(0, 0.25))
            if i == 8:
                # a relay restart between PRE and POST, the POST after it: received
                n.relay.signal(signal.SIGTERM)
                n.relay.proc.wait(timeout=10)
                n.start_relay()
                n.d.wait_log("connected to the event relay", count=1, timeout=10)
            n.inject(f"{gpu} 4 storm post {i}")
            time.sleep(rnd.uniform(0, 0.25))
        deadline = time.time() + 20
        h = n.rewatch()
        while h != ["Healthy", "Healthy"]:
            assert time.time() < deadline, (h, n.d.log()[-4000:])
            try:
                h = n.health(timeout=1)
            except Exception:
                h = n.rewatch()
        dlog = n.d.log()
        assert dlog.count("received SIGHUP") >= 8  # (SIGHUPs sent while one is pending coalesce)
        assert "recovered without GPU_POST_RESET" not in dlog
        rlog = n.relay.log()
        assert "re-enumerating" not in rlog, rlog
    finally:
        n.stop()


def test_a_restarted_plugin_container_resumes_the_relays_stream(scratch):
    """With --health-state-file the daemon's place in the relay's event stream
    (<state>.relay) outlives the process: a plugin container restarted between
    a GPU's PRE_RESET and POST_RESET gets the POST_RESET replayed by the relay
    -- which kept running and held it -- and the GPU is Healthy at once, not
    after the polled hold (set out of reach). Without the file the new process
    starts a gap (tested above)."""
    state = os.path.join(scratch + ".fixture", "health.state")
    n = RelayNode(scratch, daemon_args=["--health-state-file", state, "--reset-recovery-hold-ms", "600000"])
    try:
        n.d.wait_log("events on through the relay")
        n.inject("1 3 mode1 reset")
        assert n.health() == ["Healthy", "Unhealthy"]
        n.call.cancel()
        n.c.close()
        assert n.d.stop() == 0
        assert open(state + ".relay").read().startswith("adp-relay-cursor v1\n")
        n.inject("1 4 reset done")  # while no daemon is connected: the relay holds it
        n.relay.wait_log(" type=4 ")
        n.d = harness.Daemon(scratch, n.fx, args=["--health-event-socket", n.sock, "--health-state-file", state,
                                                  "--reset-recovery-hold-ms", "600000"],
                             env={"LD_PRELOAD": _preload(SIM), "DP_HEALTH_POLL_MS": "200"}).start()
        first = n.rewatch()
        assert first[1] == "Unhealthy" or first == ["Healthy", "Healthy"]  # the ledger's verdict, then the replay
        if first != ["Healthy", "Healthy"]:
            n.wait_health(["Healthy", "Healthy"], timeout=5)
        assert "relay cursor " + state + ".relay: relay " in n.d.log()
        rlog = n.relay.wait_log("replaying 1 event(s)")
        assert rlog.count("daemon connected for events (nothing missed)") == 1
        assert "across an event gap" not in n.d.log()
    finally:
        n.stop()


def test_relay_exits_with_a_renewal_stuck_in_amdsmi(scratch):
    """A daemon's reinit starts a renewal just as the amdsmi event wait hangs:
    the renewal waits for the waiter, which does not return. SIGTERM then ends
    the relay after its watchdog's threshold (plus a second), not when amdsmi
    lets go: a container that would not stop is killed by the kubelet only
    after the grace period, with the node's events off all that time."""
    import socket
    n = RelayNode(scratch, relay_env={"ADP_RELAY_STUCK_MS": "1500"})
    try:
        n.d.wait_log("events on through the relay")
        n.inject("hang 8000")
        time.sleep(0.3)  # the waiter has taken the hang
        c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        c.settimeout(5)
        c.connect(n.sock)
        assert c.recv(4096).startswith(b"hello v1 ")
        c.sendall(b"reinit fp=0000000000000000\n")  # processors the registration does not have
        n.relay.wait_log("re-enumerating (a daemon asked")
        t0 = time.time()
        n.relay.signal(signal.SIGTERM)
        rc = n.relay.proc.wait(timeout=10)
        took = time.time() - t0
        c.close()
        assert rc == 0, rc
        log = n.relay.log()
        assert "exiting with a registration renewal stuck in amdsmi" in log, log[-3000:]
        assert took < 5.0, took  # 1.5 s watchdog + 1 s, not the 8 s hang
    finally:
        n.stop()


def test_a_relay_that_never_answers_the_reinit_is_a_gap(scratch, tmp_path):
    """A relay that greets but never answers the daemon's reinit (its
    registrar stuck): after ADP_EVENT_FAIL_MS the daemon polls, records an
    event gap, and a GPU that was waiting for GPU_POST_RESET recovers by the
    polled check."""
    import socket
    import threading
    sock = str(tmp_path / "mute.sock")
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(sock)
    srv.listen(4)
    conns = []
    stop = threading.Event()

    def serve():
        srv.settimeout(0.2)
        while not stop.is_set():
            try:
                conn, _ = srv.accept()
            except OSError:
                continue
            conn.sendall(b"hello v1 events=ok processors=2 relay=00ab gen=1 seq=0 fp=- renew_ms=1\n")
            conns.append(conn)  # read nothing, answer nothing
    t = threading.Thread(target=serve, daemon=True)
    t.start()
    fx = fixtures.node(2)
    state = tmp_path / "health.state"
    state.write_text(f"adp-health v1\n{fx['gpus'][1]['uuid']}\t-\t0\t4\tGPU_PRE_RESET: seeded\n")
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, args=["--health-event-socket", sock, "--health-state-file", str(state),
                                          "--reset-recovery-hold-ms", "500"],
                       env={"DP_HEALTH_POLL_MS": "100", "ADP_EVENT_FAIL_MS": "700"}).start()
    try:
        log = d.wait_log("has not answered this daemon's reinit for 700 ms")
        assert "events on through the relay" not in log
        log = d.wait_log("recovered without GPU_POST_RESET", timeout=10)
        assert "no GPU_POST_RESET after an event gap (the event relay did not answer)" in log, log[-3000:]
    finally:
        d.stop()
        k.stop()
        stop.set()
        t.join(5)
        for c in conns:
            c.close()
        srv.close()


def test_a_dropped_connection_is_a_tentative_gap_the_replay_cancels(scratch):
    """The relay drops a daemon whose socket buffer is full (here: on cue,
    ADP_DEBUG_RELAY_DROP_ON). The GPU waiting for GPU_POST_RESET gets a
    *tentative* gap: the daemon reconnects with its cursor, the relay replays
    what it missed and says nothing was lost, and the mark is cancelled -- so
    polling does not return the GPU (the hold passes several times over), and
    the POST_RESET replayed or sent later does. A POST_RESET the drop itself
    swallowed arrives by the replay."""
    n = RelayNode(scratch, relay_env={"ADP_DEBUG_RELAY_DROP_ON": "dropme"},
                  daemon_args=["--reset-recovery-hold-ms", "500"])
    try:
        n.d.wait_log("events on through the relay")
        n.inject("1 3 pre-reset")
        assert n.health() == ["Healthy", "Unhealthy"]
        # a VMFAULT on GPU 0 whose delivery drops the connection
        n.inject("0 1 fault dropme")
        n.d.wait_log("event relay: the event relay closed the connection")
        log = n.d.wait_log("the event relay replayed what was missed; waiting for GPU_POST_RESET again", timeout=10)
        assert n.bdf(1) in log
        assert "VMFAULT(1) on GPU 0" in n.d.wait_log("VMFAULT(1) on GPU 0")  # replayed
        time.sleep(1.5)  # three holds: no polled recovery without a real gap
        assert "recovered without GPU_POST_RESET" not in n.d.log()
        assert _series(n.metrics(), "amdgpu_dp_gpu_awaiting_polled_recovery", n.bdf(1)) == 0
        # the POST_RESET whose delivery drops the connection arrives by the replay
        n.inject("1 4 reset done dropme")
        n.d.wait_log("event relay: the event relay closed the connection", count=2)
        n.wait_health(["Healthy", "Healthy"], timeout=10)
        rlog = n.relay.log()
        assert rlog.count("daemon connected for events (nothing missed)") == 2, rlog[-3000:]
        assert "recovered without GPU_POST_RESET" not in n.d.log()
    finally:
        n.stop()


def test_an_event_the_relay_itself_dropped_is_a_confirmed_gap(scratch):
    """The relay's waiter cannot hand an event to its poll loop (the pipe
    between them full; here on cue, ADP_DEBUG_RELAY_REFUSE_EVENT): the event is
    in no daemon's stream and in no replay. The relay tells every daemon it may
    have missed events, and the GPU waiting for that GPU_POST_RESET comes back
    by the polled recovery instead of staying Unhealthy. Events after the loss
    are delivered as before."""
    n = RelayNode(scratch, relay_env={"ADP_DEBUG_RELAY_REFUSE_EVENT": "lostme"},
                  daemon_args=["--reset-recovery-hold-ms", "500"])
    try:
        n.d.wait_log("events on through the relay")
        n.inject("1 3 pre-reset")
        assert n.health() == ["Healthy", "Unhealthy"]
        n.inject("1 4 reset done lostme")
        rlog = n.relay.wait_log("event(s) lost after #1: daemons are told they may have missed events")
        assert "event dropped (relay loop behind)" in rlog
        log = n.d.wait_log("across an event gap", timeout=10)
        assert n.bdf(1) in log
        n.wait_health(["Healthy", "Healthy"], timeout=10)
        line = [ln for ln in n.d.log().splitlines() if "recovered without GPU_POST_RESET" in ln]
        assert len(line) == 1 and n.bdf(1) in line[0], line
        assert "GPU_POST_RESET(4)" not in n.d.log()  # it never arrived
        # A daemon reconnecting with a cursor at the loss may have missed it ...
        n.d.signal(signal.SIGHUP)
        assert n.rewatch() == ["Healthy", "Healthy"]
        n.relay.wait_log("daemon connected for events (it may have missed events)")
        n.d.wait_log("events on through the relay", count=2)
        # ... one whose cursor is past it has not; events flow as before.
        n.inject("0 3 pre-reset")
        n.wait_health(["Unhealthy", "Healthy"], timeout=10)
        n.d.signal(signal.SIGHUP)
        assert n.rewatch() == ["Unhealthy", "Healthy"]
        n.relay.wait_log("daemon connected for events (nothing missed)")
        n.d.wait_log("events on through the relay", count=3)
        n.inject("0 4 reset done")
        n.wait_health(["Healthy", "Healthy"], timeout=10)
    finally:
        n.stop()


def test_a_relay_gone_for_good_confirms_the_gap(scratch):
    """The relay dies and does not come back: the tentative gap of the GPU
    waiting for GPU_POST_RESET is confirmed after ADP_EVENT_FAIL_MS without a
    relay, and the polled recovery returns the GPU. Before that, nothing
    returns it (a relay that came back could still replay the event)."""
    n = RelayNode(scratch, daemon_args=["--reset-recovery-hold-ms", "300"],
                  daemon_env={"ADP_EVENT_FAIL_MS": "1500"})
    try:
        n.d.wait_log("events on through the relay")
        n.inject("1 3 pre-reset")
        assert n.health() == ["Healthy", "Unhealthy"]
        t0 = time.time()
        n.relay.proc.kill()
        n.relay.proc.wait(timeout=10)
        log = n.d.wait_log("events may have been missed")
        assert n.bdf(1) in log
        assert _series(n.metrics(), "amdgpu_dp_gpu_awaiting_polled_recovery", n.bdf(1)) == 0  # tentative
        log = n.d.wait_log("the event relay has been unreachable for 1.5 s", timeout=10)
        n.wait_health(["Healthy", "Healthy"], timeout=10)
        assert time.time() - t0 >= 1.5
        line = [ln for ln in n.d.log().splitlines() if "recovered without GPU_POST_RESET" in ln]
        assert len(line) == 1 and "unreachable" in line[0], line
    finally:
        n.stop()


import pytest  # noqa: E402


@pytest.mark.parametrize("seed", [int(s) for s in os.environ.get("ADP_CHAOS_SEEDS", "11,12,13").split(",")])
def test_chaos_of_resets_restarts_and_drops_leaves_no_gpu_stuck(scratch, seed):
    """A seeded random mix of everything that can come between a GPU_PRE_RESET
    and its GPU_POST_RESET: daemon SIGHUPs, the relay dropping the daemon (its
    buffer full: ADP_DEBUG_RELAY_DROP_ON), a POST_RESET the relay itself loses
    (ADP_DEBUG_RELAY_REFUSE_EVENT), the relay restarted (SIGTERM or SIGKILL),
    events in between. Every POST_RESET is sent while a relay runs;
    it reaches the daemon directly or by the relay's replay -- unless the relay
    lost it, or the relay holding it restarts before the daemon is back; the
    daemon sees either as an event gap: then the polled check returns the GPU. Either
    way no GPU stays out of service, and a polled return only ever follows a
    confirmed gap on that GPU."""
    import random
    rnd = random.Random(seed)
    n = RelayNode(scratch, relay_env={"ADP_DEBUG_RELAY_DROP_ON": "dropme", "ADP_DEBUG_RELAY_REFUSE_EVENT": "lostme"},
                  daemon_args=["--reset-recovery-hold-ms", "1500", "--reset-flap-limit", "0"])
    try:
        n.d.wait_log("events on through the relay")
        pending = set()
        for i in range(24):
            op = rnd.choice(["pre", "post", "post", "sighup", "drop", "restart", "vm"])
            gpu = rnd.randrange(2)
            if op == "pre":
                n.inject(f"{gpu} 3 chaos pre {i}")
                pending.add(gpu)
            elif op == "post" and pending:
                g = rnd.choice(sorted(pending))
                # dropme: the relay drops the daemon (the replay brings it);
                # lostme: the relay's own waiter drops it (a confirmed gap)
                n.inject(f"{g} 4 chaos post {i}" + rnd.choice(["", "", " dropme", " dropme", " lostme"]))
                pending.discard(g)
            elif op == "sighup":
                n.d.signal(signal.SIGHUP)
            elif op == "drop":
                n.inject(f"{gpu} 1 chaos vm dropme {i}")
            elif op == "restart":
                if rnd.random() < 0.5:
                    n.relay.signal(signal.SIGTERM)
                else:
                    n.relay.proc.kill()
                n.relay.proc.wait(timeout=10)
                n.start_relay()
            elif op == "vm":
                n.inject(f"{gpu} 1 chaos vm {i}")
            time.sleep(rnd.uniform(0, 0.15))
        for g in sorted(pending):
            n.inject(f"{g} 4 chaos final post {g}")
        # The plugin's socket name never changes: watch it afresh until the
        # node is Healthy (a SIGHUP may restart the plugin under a watch).
        endpoint = os.path.join(scratch, n.k.wait_registration(10).endpoint)
        deadline = time.time() + 20
        h = None
        while h != ["Healthy", "Healthy"]:
            if time.time() >= deadline and os.environ.get("ADP_CHAOS_DUMP"):
                open(os.environ["ADP_CHAOS_DUMP"] + ".daemon", "w").write(n.d.log())
                import glob
                with open(os.environ["ADP_CHAOS_DUMP"] + ".relays", "w") as f:
                    for r in sorted(glob.glob(scratch + "-relay*.daemon.log")):
                        f.write(f"==== {r}\n" + open(r).read())
            assert time.time() < deadline, (seed, h, n.d.log()[-5000:])
            try:
                c = kubelet.PluginClient(endpoint)
                q, call = c.watch()
                try:
                    while h != ["Healthy", "Healthy"] and time.time() < deadline:
                        h = [x.health for x in q.get(timeout=1).devices]
                finally:
                    call.cancel()
                    c.close()
            except Exception:
                time.sleep(0.2)
        log = n.d.log().splitlines()
        for i, ln in enumerate(log):
            if "recovered without GPU_POST_RESET" in ln:
                bdf = ln.split("GPU ")[1].split(" ")[0]
                assert any(f"GPU {bdf} waits for GPU_POST_RESET across an event gap" in p for p in log[:i]), ln
    finally:
        n.stop()


def test_a_gap_confirmed_before_a_container_restart_still_ends_the_wait(scratch):
    """GPU_PRE_RESET, then the relay restarts mid-reset (its POST_RESET is
    lost: a confirmed gap), then the plugin container restarts before the
    polled hold has passed. The new process connects to the same relay with its
    cursor and misses nothing from there on -- but the gap is in the state file,
    so the polled check still returns the GPU (without it, the GPU would wait
    for a POST_RESET that will never come)."""
    state = os.path.join(scratch + ".fixture", "health.state")
    args = ["--health-state-file", state, "--reset-recovery-hold-ms", "1500"]
    n = RelayNode(scratch, daemon_args=args)
    try:
        n.d.wait_log("events on through the relay")
        n.inject("1 3 mode1 reset")
        assert n.health() == ["Healthy", "Unhealthy"]
        n.relay.proc.kill()
        n.relay.proc.wait(timeout=10)
        n.start_relay()
        n.d.wait_log("waits for GPU_POST_RESET across an event gap")
        line = [ln for ln in open(state).read().splitlines() if ln.startswith(n.fx["gpus"][1]["uuid"])][0]
        assert "\tgap=" in line, line
        n.call.cancel()
        n.c.close()
        assert n.d.stop() == 0  # before the hold has passed
        assert "recovered without GPU_POST_RESET" not in n.d.log()
        n.d = harness.Daemon(scratch, n.fx, args=["--health-event-socket", n.sock, *args],
                             env={"LD_PRELOAD": _preload(SIM), "DP_HEALTH_POLL_MS": "200"}).start()
        first = n.rewatch()
        assert first == ["Healthy", "Unhealthy"], first
        log = n.d.wait_log("across an event gap from before this process")
        assert n.bdf(1) in log
        n.relay.wait_log("daemon connected for events (nothing missed)")  # its own link missed nothing
        assert n.wait_health(["Healthy", "Healthy"], timeout=10) == ["Healthy", "Healthy"]
        assert "recovered without GPU_POST_RESET" in n.d.log()
        line = [ln for ln in open(state).read().splitlines() if ln.startswith(n.fx["gpus"][1]["uuid"])][0]
        assert "gap=" not in line and line.split("\t")[3] == "0", line
    finally:
        n.stop()

"""Health pipeline: amdsmi events / RAS polling -> ListAndWatch updates, with recovery.

Parity: reference nvidia.go:181-294 (checkHealth, DP_DISABLE_HEALTHCHECKS,
application-error ignore list), server.go:251-265 (ListAndWatch resend).
Fault injection goes through the amdsmi mock's event FIFO and state directory.
Fixes pinned here: B1 (health reaches every replica), B15 (recovery).
"""

import os
import time

import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet, native

# nvidia_test.go:31-64 TestGetAdditionalXids, same semantics for amdsmi event IDs.
XID_CASES = [("", []), (",", []), ("not-an-int", []), ("68", [68]), ("-68", []), ("68  ", [68]),
             ("68,", [68]), (",68", [68]), ("68,67", [68, 67]), ("68,not-an-int,67", [68, 67])]


@pytest.mark.parametrize("text,want", XID_CASES)
def test_additional_ids_reference_vectors(text, want):
    assert native.parse_additional_ids(text) == want


def test_event_classification():
    c = native.health_config("", "")
    assert not c["disabled"]
    v = c["verdicts"]
    assert v["3"] == -1  # GPU_PRE_RESET -> unhealthy
    assert v["4"] == +1  # GPU_POST_RESET -> healthy (recovery)
    assert v["1"] == 0 and v["2"] == 0  # VMFAULT / THERMAL_THROTTLE: application events, ignored
    assert native.health_config("all", "")["disabled"]
    assert native.health_config("xids", "")["disabled"]
    assert native.health_config("foo,XIDS", "")["disabled"]
    c = native.health_config("3", "0")
    assert c["verdicts"]["3"] == 0 and c["poll_ms"] == 0


class Node:
    def __init__(self, scratch, fx, env=None, args=()):
        self.fifo = os.path.join(scratch + ".fixture", "events")
        self.state = os.path.join(scratch + ".fixture", "state")
        os.makedirs(self.state, exist_ok=True)
        os.mkfifo(self.fifo)
        self.k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        self.d = harness.Daemon(scratch, fx, args=args, env=env, event_fifo=self.fifo,
                                state_dir=self.state).start()
        reg = self.k.wait_registration()
        self.c_path = os.path.join(scratch, reg.endpoint)
        self.c = kubelet.PluginClient(self.c_path)
        self.q, self.call = self.c.watch()
        self.first = self.q.get(timeout=5)
        # The monitor starts after registration (reference server.go:148): wait until
        # it has taken its ECC baselines and registered for events.
        disabled = (env or {}).get("DP_DISABLE_HEALTHCHECKS", "").lower()
        self.d.wait_log("health checks disabled" if disabled in ("all", "xids") else "health monitor watching")

    def inject(self, line, reader=True):
        # The health thread opens the FIFO when it registers for events, which can
        # come after the first ListAndWatch: wait for it unless none is expected.
        deadline = time.monotonic() + (5 if reader else 0)
        while True:
            try:
                fd = os.open(self.fifo, os.O_WRONLY | os.O_NONBLOCK)
                break
            except OSError as e:
                if e.errno != 6:  # ENXIO: no reader (yet, or health checks disabled)
                    raise
                if time.monotonic() >= deadline:
                    assert not reader, "health thread never opened the event FIFO"
                    return
                time.sleep(0.02)
        os.write(fd, (line + "\n").encode())
        os.close(fd)

    def next(self, timeout=5):
        return self.q.get(timeout=timeout)

    def health(self, resp):
        return {x.ID: x.health for x in resp.devices}

    def close(self):
        self.call.cancel()
        self.c.close()
        code = self.d.stop()
        self.k.stop()
        return code


@pytest.fixture
def node(scratch):
    nodes = []

    def make(fx=None, **kw):
        n = Node(scratch, fx or fixtures.node(2), **kw)
        nodes.append(n)
        return n
    yield make
    for n in nodes:
        n.close()


def test_reset_marks_unhealthy_then_recovers(node):
    n = node()
    ids = [x.ID for x in n.first.devices]
    n.inject("0 3 pre-reset")
    h = n.health(n.next())
    assert h == {ids[0]: "Unhealthy", ids[1]: "Healthy"}
    n.inject("0 4 post-reset")
    h = n.health(n.next())
    assert h == {ids[0]: "Healthy", ids[1]: "Healthy"}


def test_application_events_are_ignored(node):
    n = node()
    n.inject("1 1 vm fault")
    n.inject("1 2 thermal")
    deadline = time.monotonic() + 5
    while n.d.log().count("(ignored; ") < 2 and time.monotonic() < deadline:
        time.sleep(0.05)
    assert n.d.log().count("(ignored; ") >= 2
    time.sleep(0.3)
    assert n.q.empty()


def test_a_storm_of_ignored_events_is_counted_not_logged_line_by_line(node):
    """A workload that faults in a loop sends VM faults by the thousand: each is
    counted (amdgpu_dp_gpu_events_total), the log gets the first ten and then
    every thousandth, and health does not change."""
    n = node(args=["--metrics-addr", "127.0.0.1:0"])
    import re
    from test_metrics import _get, _parse
    port = int(re.search(r"on port (\d+)", n.d.wait_log("serving /metrics")).group(1))
    for i in range(0, 2500, 250):
        n.inject("".join(f"1 1 vm fault {i + j}\n" for j in range(250)).rstrip("\n"))
    deadline = time.monotonic() + 15
    total = 0
    while time.monotonic() < deadline:
        m = _parse(_get(port, "/metrics")[1])
        total = sum(v for (name, ls), v in m.items()
                    if name == "amdgpu_dp_gpu_events_total" and dict(ls).get("type") == "VMFAULT")
        if total >= 2500:
            break
        time.sleep(0.1)
    assert total == 2500, total
    lines = [ln for ln in n.d.log().splitlines() if "VMFAULT(1)" in ln]
    assert len(lines) == 12, len(lines)  # 1..10, 1000th, 2000th
    assert "(ignored; 2000 of this type so far)" in lines[-1]
    assert n.q.empty()


def test_health_reaches_every_replica(node):
    # Reference defect B1: Unhealthy was set on the raw device, never the advertised replicas.
    n = node(args=["--resource-config", "gpu:sharedgpu:3"])
    assert len(n.first.devices) == 6
    n.inject("1 3")
    h = n.next()
    bad = sorted(x.ID for x in h.devices if x.health == "Unhealthy")
    assert len(bad) == 3 and all("-replica-" in i for i in bad)
    assert len({i.split("-replica-")[0] for i in bad}) == 1


def test_partition_reset_takes_down_the_whole_gpu(node):
    n = node(fixtures.node(2, "CPX", memory="NPS2"), args=["--partition-strategy", "single"])
    assert len(n.first.devices) == 16
    n.inject("1:5 3")  # reset seen on partition 5 of GPU 1
    h = n.next()
    assert sum(x.health == "Unhealthy" for x in h.devices) == 8


def test_disable_healthchecks_ignores_configured_ids(node):
    n = node(env={"DP_DISABLE_HEALTHCHECKS": "3"})
    n.inject("0 3")
    time.sleep(0.8)
    assert n.q.empty()


def test_disable_all(node):
    n = node(env={"DP_DISABLE_HEALTHCHECKS": "all"})
    n.inject("0 3", reader=False)
    time.sleep(0.8)
    assert n.q.empty()
    assert "health checks disabled" in n.d.log()


def test_ecc_polling(node):
    n = node(env={"DP_HEALTH_POLL_MS": "100"})
    ids = [x.ID for x in n.first.devices]
    with open(os.path.join(n.state, "gpu1.ecc"), "w") as f:
        f.write("7\n")
    h = n.health(n.next())
    assert h[ids[1]] == "Unhealthy" and h[ids[0]] == "Healthy"
    n.inject("1 4")  # a completed reset clears it
    assert n.health(n.next())[ids[1]] == "Healthy"


def test_unresponsive_device_recovers(node):
    n = node(env={"DP_HEALTH_POLL_MS": "100"})
    ids = [x.ID for x in n.first.devices]
    dead = os.path.join(n.state, "gpu0.dead")
    open(dead, "w").close()
    assert n.health(n.next())[ids[0]] == "Unhealthy"
    os.unlink(dead)
    assert n.health(n.next())[ids[0]] == "Healthy"


def test_events_unsupported_falls_back_to_polling(node):
    fx = fixtures.node(2)
    fx["events_supported"] = False
    n = node(fx, env={"DP_HEALTH_POLL_MS": "100"})
    assert all(x.health == "Healthy" for x in n.first.devices)  # not marked unhealthy
    assert "using polling only" in n.d.log()
    open(os.path.join(n.state, "gpu0.dead"), "w").close()
    assert "Unhealthy" in n.health(n.next()).values()


def test_every_watcher_on_every_loop_sees_each_transition(node):
    """Watchers are spread over the server's loops; one transition reaches each once."""
    n = node(args=["--server-threads", "4"])
    ids = [x.ID for x in n.first.devices]
    extra = []
    for _ in range(7):  # 8 connections over 4 loops (+ the self-dial probe)
        c = kubelet.PluginClient(n.c_path)
        q, call = c.watch()
        assert n.health(q.get(timeout=5)) == {i: "Healthy" for i in ids}
        extra.append((c, q, call))
    n.inject("1 3")
    for q in [n.q] + [e[1] for e in extra]:
        assert n.health(q.get(timeout=5))[ids[1]] == "Unhealthy"
    time.sleep(0.3)
    assert all(q.empty() for q in [n.q] + [e[1] for e in extra])  # no duplicates
    for c, _, call in extra:
        call.cancel()
        c.close()


def test_events_counted_per_gpu_and_type_on_metrics(node):
    """Every amdsmi event is counted per GPU and type on /metrics, ignored ones
    too: an application's VM faults and thermal throttling never change health,
    but an operator wants to see them (amdgpu_dp_gpu_events_total)."""
    import re
    import urllib.request
    n = node(args=["--metrics-addr", "127.0.0.1:0"])
    port = int(re.search(r"serving /metrics and /healthz on port (\d+)",
                         n.d.wait_log("serving /metrics and /healthz on port")).group(1))
    bdfs = [g["bdf"] for g in fixtures.node(2)["gpus"]]
    for line in ("1 1 vm fault", "1 1 vm fault", "1 2 thermal", "0 3 pre-reset", "0 4 post-reset"):
        n.inject(line)
    want = {(bdfs[1], "VMFAULT"): 2, (bdfs[1], "THERMAL_THROTTLE"): 1, (bdfs[0], "GPU_PRE_RESET"): 1,
            (bdfs[0], "GPU_POST_RESET"): 1}
    deadline = time.monotonic() + 5
    while True:
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
        got = {}
        for ln in body.splitlines():
            if ln.startswith("amdgpu_dp_gpu_events_total{"):
                labels = dict(kv.split("=", 1) for kv in ln[ln.index("{") + 1:ln.index("}")].split(","))
                got[(labels["bdf"].strip('"'), labels["type"].strip('"'))] = int(ln.split()[-1])
        if got == want or time.monotonic() > deadline:
            break
        time.sleep(0.05)
    assert got == want, body[-2000:]


def test_healthz_fails_while_the_health_loop_is_stuck(scratch):
    """A health monitor stuck in a call that does not return (here the mock's
    event wait, "hang") stops its loop: /healthz answers 503 -- the liveness
    probe restarts the daemon -- and 200 again once the loop moves.
    amdgpu_dp_health_loop_age_seconds shows the age."""
    import re
    from test_metrics import _get, _parse, _value
    n = Node(scratch, dict(fixtures.node(1), events_open_kfd=True), args=["--metrics-addr", "127.0.0.1:0"],
             env={"ADP_HEALTH_STALL_MS": "400", "DP_HEALTH_POLL_MS": "100"})
    try:
        port = int(re.search(r"on port (\d+)", n.d.wait_log("serving /metrics")).group(1))
        assert _get(port, "/healthz")[0] == 200
        assert _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_health_loop_age_seconds") < 0.4
        n.inject("hang 2000")
        deadline = time.time() + 3
        while _get(port, "/healthz")[0] != 503:
            assert time.time() < deadline
            time.sleep(0.05)
        assert _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_health_loop_age_seconds") > 0.4
        assert "the health monitor has not advanced for" in n.d.log()
        deadline = time.time() + 5
        while _get(port, "/healthz")[0] != 200:
            assert time.time() < deadline
            time.sleep(0.05)
    finally:
        n.close()


def test_failing_event_waits_report_events_off_until_they_succeed(scratch):
    """In-process events: amdsmi event waits that keep failing (the mock's
    "fail <n>") deliver nothing, so after ADP_EVENT_FAIL_MS the daemon reports
    events off (amdgpu_dp_health_events_enabled 0) and logs it once, not every
    100 ms; when waits succeed again events are on and reset events work."""
    import re
    from test_metrics import _get, _parse, _value
    n = Node(scratch, dict(fixtures.node(2), events_open_kfd=True), args=["--metrics-addr", "127.0.0.1:0"],
             env={"ADP_EVENT_FAIL_MS": "300"})
    try:
        port = int(re.search(r"on port (\d+)", n.d.wait_log("serving /metrics")).group(1))

        def enabled():
            return _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_health_events_enabled")
        assert enabled() == 1
        n.inject("fail 20")
        deadline = time.time() + 5
        while enabled() != 0:
            assert time.time() < deadline
            time.sleep(0.05)
        assert "events off, polling only until they succeed" in n.d.log()
        n.d.wait_log("amdsmi event waits succeed again: events on", timeout=10)
        assert enabled() == 1
        assert n.d.log().count("event wait failed (") == 1  # rate-limited
        n.inject("1 3 mode1 reset")
        assert [x.health for x in n.next().devices] == ["Healthy", "Unhealthy"]
    finally:
        n.close()


def test_operator_drain_file(scratch, tmp_path):
    """--drain-file: a GPU named in it (PCI address, UUID, node index; '#'
    comments) is advertised Unhealthy -- every replica of it -- until removed;
    a GPU_POST_RESET does not undo a drain."""
    import queue
    drain = tmp_path / "drain"
    fx = dict(fixtures.node(2), events_open_kfd=True)
    n = Node(scratch, fx, args=["--resource-config", "gpu:sharedgpu:2", "--drain-file", str(drain),
                                "--metrics-addr", "127.0.0.1:0"], env={"DP_HEALTH_POLL_MS": "100"})
    try:
        last = [x.health for x in n.first.devices]

        def until(want, timeout=5):
            nonlocal last
            deadline = time.time() + timeout
            while last != want and time.time() < deadline:
                try:
                    last = [x.health for x in n.q.get(timeout=0.2).devices]
                except queue.Empty:
                    pass
            return last
        drain.write_text(f"# maintenance\n{fx['gpus'][1]['bdf']}  # bad fan\n")
        assert until(["Healthy", "Healthy", "Unhealthy", "Unhealthy"]) == ["Healthy", "Healthy", "Unhealthy",
                                                                          "Unhealthy"]
        assert "drained by the operator" in n.d.wait_log("drained by the operator")
        import re
        from test_metrics import _get, _parse, _value
        port = int(re.search(r"on port (\d+)", n.d.log()).group(1))
        m = _parse(_get(port, "/metrics")[1])
        bdf1 = fx["gpus"][1]["bdf"]
        assert _value(m, "amdgpu_dp_gpu_failure", bdf=bdf1, cause="drained") == 1
        assert _value(m, "amdgpu_dp_gpu_failure", bdf=bdf1, cause="ecc") == 0
        assert _value(m, "amdgpu_dp_gpu_failure", bdf=fx["gpus"][0]["bdf"], cause="drained") == 0
        import subprocess
        import sys
        st = subprocess.run([sys.executable, "-m", "k8s_gpu_sharing_plugin_amd", "status",
                             f"http://127.0.0.1:{port}/metrics"], capture_output=True, text=True, timeout=60)
        assert f"GPU {bdf1}: drained" in st.stdout and st.returncode == 1, st.stdout
        n.inject("1 4 reset done")  # a post-reset clears faults, not a drain
        n.d.wait_log("GPU_POST_RESET")
        time.sleep(0.4)
        assert until(["Healthy"] * 4, timeout=0.5) == ["Healthy", "Healthy", "Unhealthy", "Unhealthy"]
        drain.write_text("0\n")  # node index 0 instead
        assert until(["Unhealthy", "Unhealthy", "Healthy", "Healthy"]) == ["Unhealthy", "Unhealthy", "Healthy",
                                                                          "Healthy"]
        drain.unlink()
        assert until(["Healthy"] * 4) == ["Healthy"] * 4
    finally:
        n.close()


def test_a_partition_pci_function_drains_its_gpu(scratch, tmp_path):
    """On a CPX node amd-smi lists each compute partition with its own PCI
    function (0000:2c:00.0 .. .7): naming any of them in the drain file drains
    the whole GPU -- all 8 partitions -- as a reset holds it."""
    import queue
    drain = tmp_path / "drain"
    fx = fixtures.node(2, modes="CPX")
    n = Node(scratch, fx, args=["--partition-strategy", "single", "--drain-file", str(drain)],
             env={"DP_HEALTH_POLL_MS": "100"})
    try:
        drain.write_text(fx["gpus"][1]["bdf"][:-1] + "3  # a partition of GPU 1\n")
        deadline = time.time() + 5
        bad = 0
        while bad != 8 and time.time() < deadline:
            try:
                bad = sum(x.health != "Healthy" for x in n.q.get(timeout=0.2).devices)
            except queue.Empty:
                pass
        assert bad == 8
        n.d.wait_log("drained by the operator")
    finally:
        n.close()


def test_drain_and_undrain_commands(scratch, tmp_path):
    """`amdgpu-device-plugin --drain <id>` / `--undrain <id>` (run in the
    plugin pod, DP_DRAIN_FILE set) edit the drain file -- IDs checked against
    this node's GPUs -- and the running daemon applies it at its next poll."""
    import queue
    import subprocess
    from k8s_gpu_sharing_plugin_amd import DAEMON, MOCK_LIB
    drain = tmp_path / "drain"
    fx = dict(fixtures.node(2), events_open_kfd=True)
    n = Node(scratch, fx, args=["--drain-file", str(drain)], env={"DP_HEALTH_POLL_MS": "100"})
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=fixtures.write(fx, str(tmp_path / "fx")),
               DP_DRAIN_FILE=str(drain))

    def cli(*args):
        r = subprocess.run([DAEMON, "--device-plugin-path", str(tmp_path), *args], capture_output=True, text=True,
                           timeout=60, env=env)
        return r.returncode, r.stdout, r.stderr

    last = [x.health for x in n.first.devices]

    def until(want, timeout=5):
        nonlocal last
        deadline = time.time() + timeout
        while last != want and time.time() < deadline:
            try:
                last = [x.health for x in n.q.get(timeout=0.2).devices]
            except queue.Empty:
                pass
        return last
    try:
        bdf1, uuid1 = fx["gpus"][1]["bdf"], fx["gpus"][1]["uuid"]
        rc, out, _ = cli("--drain", bdf1)
        assert rc == 0 and out.startswith(bdf1) and uuid1 in out, out
        assert until(["Healthy", "Unhealthy"]) == ["Healthy", "Unhealthy"]
        rc, out, _ = cli("--drain", uuid1)  # already listed under another name: unchanged
        assert rc == 0 and out.count("\n") == 1
        rc, _, err = cli("--drain", "0000:99:00.0")
        assert rc == 1 and "no GPU of this node is named 0000:99:00.0" in err
        rc, out, _ = cli("--undrain", "1")  # by node index
        assert rc == 0 and out == ""
        assert until(["Healthy", "Healthy"]) == ["Healthy", "Healthy"]
        # a hand-written line draining both GPUs: undraining one keeps the other and the comment
        bdf0 = fx["gpus"][0]["bdf"]
        drain.write_text(f"# planned work\n{bdf0},{uuid1}  # rack 4 maintenance\n")
        assert until(["Unhealthy", "Unhealthy"]) == ["Unhealthy", "Unhealthy"]
        rc, out, err = cli("--undrain", bdf1)
        assert rc == 0 and out == f"# planned work\n{bdf0}  # rack 4 maintenance\n", out
        assert "kept on the same line" in err
        assert until(["Unhealthy", "Healthy"]) == ["Unhealthy", "Healthy"]
    finally:
        n.close()


def test_return_to_service_command(scratch, tmp_path):
    """`amdgpu-device-plugin --return-to-service <id>` (in the plugin pod,
    DP_DRAIN_FILE set): the running daemon clears what it holds against the
    GPU at its next poll -- a reset that never completed, a flapping
    quarantine, an ECC verdict (re-baselined at the current count) -- as if
    its line were deleted from the state file, without a restart. A drain
    stays (that is --undrain's); a name that is no GPU of the node fails."""
    import queue
    import subprocess
    from k8s_gpu_sharing_plugin_amd import DAEMON, MOCK_LIB
    drain = tmp_path / "drain"
    state = tmp_path / "health.state"
    fx = dict(fixtures.node(2), events_open_kfd=True)
    n = Node(scratch, fx, args=["--drain-file", str(drain), "--health-state-file", str(state),
                                "--reset-recovery-hold-ms", "0", "--reset-flap-limit", "2"],
             env={"DP_HEALTH_POLL_MS": "100"})
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=fixtures.write(fx, str(tmp_path / "fx")),
               DP_DRAIN_FILE=str(drain), DP_HEALTH_POLL_MS="100")

    def cli(*args):
        r = subprocess.run([DAEMON, "--device-plugin-path", str(tmp_path), *args], capture_output=True, text=True,
                           timeout=60, env=env)
        return r.returncode, r.stdout, r.stderr

    last = [x.health for x in n.first.devices]

    def until(want, timeout=5):
        nonlocal last
        deadline = time.time() + timeout
        while last != want and time.time() < deadline:
            try:
                last = [x.health for x in n.q.get(timeout=0.2).devices]
            except queue.Empty:
                pass
        return last
    try:
        bdf0, bdf1 = fx["gpus"][0]["bdf"], fx["gpus"][1]["bdf"]
        n.d.wait_log("health poll #1")
        # GPU 1: a reset that never completes (no gap, no polled recovery)
        n.inject("1 3 pre-reset")
        assert until(["Healthy", "Unhealthy"]) == ["Healthy", "Unhealthy"]
        rc, out, err = cli("--return-to-service", bdf1)
        assert rc == 0 and bdf1 in out and "taken by the running daemon" in out, out + err
        assert until(["Healthy", "Healthy"]) == ["Healthy", "Healthy"]
        log = n.d.wait_log("returned to service by the operator")
        assert f"GPU {bdf1} returned to service by the operator (was: GPU_PRE_RESET" in log, log[-3000:]
        assert not os.path.exists(str(drain) + ".return")  # the request is consumed
        assert "\t4\t" not in state.read_text()
        # GPU 0: ECC over its baseline, and two resets (the flap limit): both cleared, the count too
        with open(os.path.join(n.state, "gpu0.ecc"), "w") as f:
            f.write("5\n")
        n.d.wait_log("uncorrectable ECC errors rose to 5")
        n.inject("0 3 pre a")
        n.inject("0 4 post a")
        n.inject("0 3 pre b")
        n.d.wait_log("quarantined")
        time.sleep(0.3)
        while not n.q.empty():  # (the POST between the resets sent a Healthy list too)
            last = [x.health for x in n.q.get_nowait().devices]
        assert last == ["Unhealthy", "Healthy"], last
        rc, _, _ = cli("--return-to-service", "0")  # by node index
        assert rc == 0
        assert until(["Healthy", "Healthy"]) == ["Healthy", "Healthy"]
        time.sleep(0.5)  # ECC re-baselined at 5: no new verdict
        while not n.q.empty():
            last = [x.health for x in n.q.get_nowait().devices]
            assert last == ["Healthy", "Healthy"], last
        assert "resets=" not in [ln for ln in state.read_text().splitlines() if ln.startswith(fx["gpus"][0]["uuid"])][0]
        n.inject("0 3 pre c")  # one reset after the return: under the limit again
        n.d.wait_log("pre c")
        assert n.d.log().count("quarantined") == 1
        # a drain stays drained
        assert cli("--drain", bdf1)[0] == 0
        assert until(["Unhealthy", "Unhealthy"]) == ["Unhealthy", "Unhealthy"]
        assert cli("--return-to-service", bdf1)[0] == 0
        n.d.wait_log(f"GPU {bdf1}: return-to-service asked: drained")
        assert last[1] == "Unhealthy"
        rc, _, err = cli("--return-to-service", "0000:99:00.0")
        assert rc == 1 and "no GPU of this node is named 0000:99:00.0" in err
    finally:
        n.close()


def test_return_to_service_without_a_daemon_says_so(tmp_path):
    """No daemon takes the request (none running, or health checks off): the
    command says so after two poll intervals (at least 2 s) and leaves the
    request queued for the next daemon."""
    import subprocess
    from k8s_gpu_sharing_plugin_amd import DAEMON, MOCK_LIB
    fx = fixtures.node(2)
    drain = tmp_path / "drain"
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=fixtures.write(fx, str(tmp_path / "fx")),
               DP_DRAIN_FILE=str(drain), DP_HEALTH_POLL_MS="100")
    t0 = time.time()
    r = subprocess.run([DAEMON, "--device-plugin-path", str(tmp_path), "--return-to-service", "0"],
                       capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0 and "the request is still waiting after 2000 ms" in r.stderr, r.stdout + r.stderr
    assert 2.0 <= time.time() - t0 < 20
    assert fx["gpus"][0]["bdf"] in open(str(drain) + ".return").read()

"""Health verdicts survive plugin restarts and daemon restarts.

Every restart trigger (SIGHUP, kubelet.sock re-creation, config-file change,
xGMI link change) builds a new plugin generation; a GPU that failed in an
earlier generation must be advertised Unhealthy by the new one from its first
ListAndWatch, and only GPU_POST_RESET (or ECC counters that a reset cleared)
brings it back. With --health-state-file the verdicts and the ECC baseline of
the first observation also survive a container restart.

Parity: the reference keeps Device health for one ListAndWatch lifetime only
(server.go:95-116,251-265; no recovery, FIXME at server.go:259) and re-reads
nothing on restart (nvidia.go:181-269); this pins the stricter behaviour.
Also here: Allocate() of an Unhealthy device (server.go:316-353 allocates it
silently) warns, or fails with --reject-unhealthy.
"""

import os
import signal
import time

import grpc
import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet


class Node:
    """Daemon on the mock (event FIFO + state dir) with a stub kubelet."""

    def __init__(self, scratch, fx=None, args=(), env=None):
        self.scratch = scratch
        fxdir = scratch + ".fixture"
        self.fifo = os.path.join(fxdir, "events")
        self.state = os.path.join(fxdir, "state")
        os.makedirs(self.state, exist_ok=True)
        if not os.path.exists(self.fifo):
            os.mkfifo(self.fifo)
        self.fx = fx or fixtures.node(2)
        self.args = list(args)
        self.env = {"DP_HEALTH_POLL_MS": "100", **(env or {})}
        self.k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        self.d = None
        self.clients = []

    def start(self):
        self.d = harness.Daemon(self.scratch, self.fx, args=self.args, env=self.env, event_fifo=self.fifo,
                                state_dir=self.state).start()
        law = self.first_law()
        # The monitor takes its ECC baselines after registration: fault injection
        # before that would become the baseline.
        disabled = self.env.get("DP_DISABLE_HEALTHCHECKS", "").lower() in ("all", "xids")
        self.d.wait_log("health checks disabled" if disabled else "health monitor watching")
        return law

    def first_law(self, timeout=10):
        reg = self.k.wait_registration(timeout)
        self.reg = reg
        c = kubelet.PluginClient(os.path.join(self.scratch, reg.endpoint))
        q, call = c.watch()
        self.clients.append((c, call))
        self.q = q
        return health(q.get(timeout=5))

    def wait_health(self, pred, timeout=5):
        deadline = time.monotonic() + timeout
        while True:
            h = health(self.q.get(timeout=max(0.05, deadline - time.monotonic())))
            if pred(h):
                return h

    def inject(self, line):
        deadline = time.monotonic() + 5
        while True:
            try:
                fd = os.open(self.fifo, os.O_WRONLY | os.O_NONBLOCK)
                break
            except OSError as e:
                if e.errno != 6 or time.monotonic() >= deadline:
                    raise
                time.sleep(0.02)
        os.write(fd, (line + "\n").encode())
        os.close(fd)

    def set_ecc(self, gpu, count):
        with open(os.path.join(self.state, f"gpu{gpu}.ecc"), "w") as f:
            f.write(f"{count}\n")

    def stop_daemon(self):
        for c, call in self.clients:
            call.cancel()
            c.close()
        self.clients = []
        code = self.d.stop() if self.d else 0
        self.d = None
        return code

    def close(self):
        code = self.stop_daemon()
        self.k.stop()
        return code


def health(resp):
    return {x.ID: x.health for x in resp.devices}


@pytest.fixture
def mk(scratch):
    nodes = []

    def make(**kw):
        n = Node(scratch, **kw)
        nodes.append(n)
        return n
    yield make
    for n in nodes:
        n.close()


def _restart_sighup(n):
    n.d.signal(signal.SIGHUP)


def _restart_kubelet(n):
    n.k.stop()
    sock = os.path.join(n.scratch, "kubelet.sock")
    if os.path.exists(sock):
        os.unlink(sock)
    n.k = kubelet.StubKubelet(sock).start()  # re-created kubelet.sock -> inotify


def _restart_config(n):
    path = os.path.join(n.scratch + ".fixture", "config.yaml")
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write("version: v1\nflags:\n  deviceIDStrategy: uuid\n  trace: true\n")
    os.rename(tmp, path)


def _restart_xgmi(n):
    with open(os.path.join(n.state, "gpu0.xgmi_down"), "w") as f:
        f.write("2\n")


TRIGGERS = {"sighup": _restart_sighup, "kubelet": _restart_kubelet, "config": _restart_config,
            "xgmi": _restart_xgmi}


@pytest.mark.parametrize("trigger", sorted(TRIGGERS))
def test_ecc_failure_survives_every_restart_trigger(mk, trigger):
    """ECC -> Unhealthy; restart; still Unhealthy from the first ListAndWatch of
    the new generation; POST_RESET -> Healthy."""
    n = mk()
    if trigger == "config":
        path = os.path.join(n.scratch + ".fixture", "config.yaml")
        with open(path, "w") as f:
            f.write("version: v1\nflags:\n  deviceIDStrategy: uuid\n")
        n.args = ["--config-file", path]
    first = n.start()
    ids = sorted(first)
    assert set(first.values()) == {"Healthy"}
    n.set_ecc(1, 7)
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    TRIGGERS[trigger](n)
    again = n.first_law(15)
    assert again == {ids[0]: "Healthy", ids[1]: "Unhealthy"}, n.d.log()[-3000:]
    assert "unhealthy since an earlier plugin generation" in n.d.log()
    # Several polls later it is still Unhealthy (the baseline was not re-taken).
    time.sleep(0.5)
    n.inject("1 4 post-reset")
    h = n.wait_health(lambda h: h[ids[1]] == "Healthy")
    assert h[ids[0]] == "Healthy"


def test_post_reset_racing_a_reregistration_leaves_the_gpu_healthy(mk):
    """GPU_POST_RESET handled while a kubelet restart re-registers the plugins:
    the new generation reads the ledger and applies its failures in one
    critical section with the health listener, so the GPU ends Healthy every
    time. ADP_DEBUG_PUBLISH_DELAY_MS holds that section open between the
    ledger read and the apply -- the window in which the reset lands."""
    n = mk(env={"ADP_DEBUG_PUBLISH_DELAY_MS": "300"}, args=["--reset-flap-limit", "0"])  # 4 resets in a row
    ids = sorted(n.start())
    for _ in range(4):
        n.inject("1 3 pre-reset")
        n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
        seen = n.d.log().count("re-registering plugins")
        _restart_kubelet(n)
        n.d.wait_log("re-registering plugins", count=seen + 1)
        time.sleep(0.1)  # inside the publish window: the failure was read, not yet applied
        n.inject("1 4 post-reset")
        law = n.first_law(15)
        if law[ids[1]] != "Healthy":
            law = n.wait_health(lambda h: h[ids[1]] == "Healthy", timeout=5)
        assert law == {ids[0]: "Healthy", ids[1]: "Healthy"}
        time.sleep(0.3)  # and it stays so
        while not n.q.empty():
            assert health(n.q.get_nowait())[ids[1]] == "Healthy"


def test_pre_reset_without_post_reset_survives_sighup(mk):
    n = mk()
    ids = sorted(n.start())
    n.inject("0 3 pre-reset")
    n.wait_health(lambda h: h[ids[0]] == "Unhealthy")
    n.d.signal(signal.SIGHUP)
    assert n.first_law() == {ids[0]: "Unhealthy", ids[1]: "Healthy"}
    n.inject("0 4 post-reset")
    n.wait_health(lambda h: h[ids[0]] == "Healthy")


def test_unresponsive_recovery_does_not_clear_pending_reset(mk):
    """A GPU that stops answering during a reset and answers again before
    GPU_POST_RESET stays Unhealthy until the POST_RESET."""
    n = mk()
    ids = sorted(n.start())
    n.inject("0 3 pre-reset")
    n.wait_health(lambda h: h[ids[0]] == "Unhealthy")
    dead = os.path.join(n.state, "gpu0.dead")
    open(dead, "w").close()
    n.d.wait_log("device not responding")
    os.unlink(dead)
    n.d.wait_log("stays unhealthy (device responding again")
    time.sleep(0.3)
    assert n.q.empty()
    n.inject("0 4 post-reset")
    n.wait_health(lambda h: h[ids[0]] == "Healthy")


def test_state_file_survives_daemon_restart(mk, scratch):
    state_file = os.path.join(scratch + ".fixture", "health.state")
    n = mk(args=["--health-state-file", state_file])
    ids = sorted(n.start())
    n.set_ecc(1, 7)
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    assert n.stop_daemon() == 0
    body = open(state_file).read()
    assert body.startswith("adp-health v1\n") and "uncorrectable ECC errors rose to 7" in body
    # A new container: the GPU is Unhealthy from the first ListAndWatch on.
    assert n.start() == {ids[0]: "Healthy", ids[1]: "Unhealthy"}
    n.d.wait_log("stays unhealthy from an earlier generation")
    # The driver cleared the RAS counters (GPU reset while the plugin was down
    # would look the same): re-baselined, Healthy again.
    n.set_ecc(1, 0)
    n.wait_health(lambda h: h[ids[1]] == "Healthy")
    assert "counters reset" in n.d.log()


def test_ecc_counters_reset_while_the_daemon_was_down(mk, scratch):
    """A GPU reset (or driver reload) while the container was down clears the
    RAS counters: the ECC failure the state file holds is gone with them. The
    monitor re-baselines at its start and the plugins (which applied the state
    file's verdicts before it started) advertise the GPU Healthy again -- no
    poll has to run for that (a poll finds nothing to change: the count it
    reads is the new baseline)."""
    state_file = os.path.join(scratch + ".fixture", "health.state")
    n = mk(args=["--health-state-file", state_file])
    ids = sorted(n.start())
    n.set_ecc(1, 7)
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    assert n.stop_daemon() == 0
    n.set_ecc(1, 2)
    n.env["DP_HEALTH_POLL_MS"] = "60000"  # the monitor's start alone, no poll
    first = n.start()
    if first[ids[1]] != "Healthy":  # the state file's verdict, published before the monitor started
        n.wait_health(lambda h: h[ids[1]] == "Healthy")
    assert "uncorrectable ECC count 2 below the 7 seen before (counters reset); re-baselined" in n.d.log()
    assert "stays unhealthy from an earlier generation" not in n.d.log()
    assert "\t2\t2\t0\t\n" in open(state_file).read()  # healthy, baseline 2, no reason
    assert "healthy again: uncorrectable ECC counters reset" in n.d.log()
    # The new baseline is the count read at start: errors after it fail the GPU again.
    assert n.stop_daemon() == 0
    n.set_ecc(1, 3)
    n.env["DP_HEALTH_POLL_MS"] = "100"
    n.start()
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    assert "rose to 3 (baseline 2)" in n.d.log()


def test_ecc_baseline_is_the_first_observation(mk, scratch):
    """Errors that accrue while the daemon is down still fail the GPU when it
    comes back (the baseline is not re-taken at each start)."""
    state_file = os.path.join(scratch + ".fixture", "health.state")
    n = mk(args=["--health-state-file", state_file])
    n.set_ecc(0, 2)
    ids = sorted(n.start())
    n.d.wait_log("health monitor watching")
    assert n.stop_daemon() == 0
    n.set_ecc(0, 5)
    first = n.start()
    assert first[ids[0]] == "Healthy"  # verdict comes from the first poll
    h = n.wait_health(lambda h: h[ids[0]] == "Unhealthy")
    assert h[ids[1]] == "Healthy"
    assert "rose to 5 (baseline 2)" in n.d.log()


def test_without_state_file_a_new_process_starts_clean(mk):
    n = mk()
    ids = sorted(n.start())
    n.set_ecc(1, 7)
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    n.stop_daemon()
    # In-memory ledger only: the new process re-baselines at 7 (documented).
    assert n.start() == {ids[0]: "Healthy", ids[1]: "Healthy"}


def test_malformed_state_file_is_ignored(mk, scratch):
    state_file = os.path.join(scratch + ".fixture", "health.state")
    os.makedirs(os.path.dirname(state_file), exist_ok=True)
    with open(state_file, "w") as f:
        f.write("something else\n")
    n = mk(args=["--health-state-file", state_file])
    assert set(n.start().values()) == {"Healthy"}
    assert "unknown format" in n.d.log()


def test_disabled_health_checks_ignore_the_ledger(mk, scratch):
    state_file = os.path.join(scratch + ".fixture", "health.state")
    n = mk(args=["--health-state-file", state_file])
    ids = sorted(n.start())
    n.set_ecc(1, 7)
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    n.stop_daemon()
    n.env["DP_DISABLE_HEALTHCHECKS"] = "all"
    assert set(n.start().values()) == {"Healthy"}


@pytest.mark.parametrize("reject", [False, True])
def test_allocate_of_unhealthy_device(mk, reject):
    n = mk(args=["--reject-unhealthy"] if reject else [])
    ids = sorted(n.start())
    n.inject("1 3 pre-reset")
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    c = n.clients[-1][0]
    assert c.allocate([ids[0]]).container_responses  # healthy: fine either way
    if reject:
        with pytest.raises(grpc.RpcError) as e:
            c.allocate([ids[1]])
        assert e.value.code() == grpc.StatusCode.FAILED_PRECONDITION
        assert ids[1] in e.value.details() and "Unhealthy" in e.value.details()
    else:
        assert c.allocate([ids[1]]).container_responses
        assert c.allocate([ids[1]]).container_responses  # a retry: counted, not logged again
        n.d.wait_log(f"device {ids[1]} is Unhealthy (allocated anyway")
        time.sleep(0.2)
        assert n.d.log().count(f"device {ids[1]} is Unhealthy (allocated anyway") == 1
    n.inject("1 4 post-reset")
    n.wait_health(lambda h: h[ids[1]] == "Healthy")
    assert c.allocate([ids[1]]).container_responses


@pytest.mark.parametrize("gate", [False, True])
def test_prestart_health_check(mk, gate):
    """--prestart-health-check: registration and GetDevicePluginOptions ask the
    kubelet for PreStartContainer, which refuses a container whose device went
    Unhealthy after admission (the kubelet retries the start); without the flag
    PreStartContainer is the reference's no-op."""
    n = mk(args=["--prestart-health-check"] if gate else [])
    ids = sorted(n.start())
    c = n.clients[-1][0]
    assert c.options().pre_start_required is gate
    assert n.reg.options.pre_start_required is gate
    c.prestart([ids[0], ids[1]])  # all healthy: fine either way
    n.inject("1 3 pre-reset")
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    c.prestart([ids[0]])
    if gate:
        with pytest.raises(grpc.RpcError) as e:
            c.prestart([ids[0], ids[1]])
        assert e.value.code() == grpc.StatusCode.FAILED_PRECONDITION and ids[1] in e.value.details()
        with pytest.raises(grpc.RpcError) as e:
            c.prestart(["no-such-device"])
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        n.d.wait_log(f"device {ids[1]} is Unhealthy; container start refused")
    else:
        c.prestart([ids[0], ids[1]])
    n.inject("1 4 post-reset")
    n.wait_health(lambda h: h[ids[1]] == "Healthy")
    c.prestart([ids[0], ids[1]])


def test_operator_clears_a_gpu_from_the_state_file_and_sighups(mk, scratch):
    """Returning a repaired GPU to service without a reset event: remove its
    line from the state file and SIGHUP; it comes back Healthy, re-baselined."""
    state_file = os.path.join(scratch + ".fixture", "health.state")
    n = mk(args=["--health-state-file", state_file])
    ids = sorted(n.start())
    n.set_ecc(1, 7)
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    lines = open(state_file).read().splitlines()
    kept = [ln for ln in lines if not ln.startswith(ids[1])]
    assert len(kept) == len(lines) - 1
    with open(state_file + ".edit", "w") as f:
        f.write("\n".join(kept) + "\n")
    os.rename(state_file + ".edit", state_file)
    n.d.signal(signal.SIGHUP)
    assert n.first_law() == {ids[0]: "Healthy", ids[1]: "Healthy"}
    n.d.wait_log(f"GPU {ids[1]} cleared by the operator")
    time.sleep(0.4)  # polls see ECC 7 = the new baseline: stays Healthy
    assert n.q.empty()
    assert "\t7\t7\t0\t" in open(state_file).read()


def test_sighup_without_edits_keeps_the_state_file_verdicts(mk, scratch):
    state_file = os.path.join(scratch + ".fixture", "health.state")
    n = mk(args=["--health-state-file", state_file])
    ids = sorted(n.start())
    n.set_ecc(0, 3)
    n.wait_health(lambda h: h[ids[0]] == "Unhealthy")
    n.d.signal(signal.SIGHUP)
    assert n.first_law() == {ids[0]: "Unhealthy", ids[1]: "Healthy"}


def test_ecc_unreadable_at_start_takes_the_first_read_as_baseline(mk):
    """A GPU whose ECC count could not be read when the monitor started is not
    failed by the first count that does read."""
    n = mk()
    ecc = os.path.join(n.state, "gpu1.ecc")
    with open(ecc, "w") as f:
        f.write("unsupported\n")  # the mock fails the query
    ids = sorted(n.start())
    n.d.wait_log("health monitor watching")
    n.set_ecc(1, 5)
    time.sleep(0.5)
    assert n.q.empty(), "first readable ECC count treated as a rise"
    n.set_ecc(1, 6)
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    assert "rose to 6 (baseline 5)" in n.d.log()


def _set_state(n, name, value):
    with open(os.path.join(n.state, name), "w") as f:
        f.write(f"{value}\n")


def test_retired_hbm_pages_past_the_threshold(mk):
    """DP_MAX_RETIRED_PAGES=5: a GPU whose driver has retired 5 HBM pages is
    Unhealthy, stays so across a restart, and comes back if the count is
    below the threshold again (e.g. a replaced board)."""
    n = mk(env={"DP_MAX_RETIRED_PAGES": "5"})
    ids = sorted(n.start())
    _set_state(n, "gpu1.badpages", 3)
    time.sleep(0.4)
    _set_state(n, "gpu1.badpages", 5)
    h = n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    assert h[ids[0]] == "Healthy"
    n.d.wait_log("5 retired HBM pages (threshold 5)")
    _restart_sighup(n)
    assert n.first_law() == {ids[0]: "Healthy", ids[1]: "Unhealthy"}  # the verdict survives the restart
    _set_state(n, "gpu1.badpages", 0)
    n.wait_health(lambda h: h[ids[1]] == "Healthy")


@pytest.mark.parametrize("readable", [True, False])
def test_retired_pages_default_to_the_drivers_threshold(mk, readable):
    """Default (-1): the driver's own bad-page threshold when amdsmi can read it
    (root); unprivileged it cannot, and retired pages are only reported."""
    n = mk()
    if readable:
        _set_state(n, "gpu0.badpage_threshold", 10)
    ids = sorted(n.start())
    n.d.wait_log("health poll #1")
    assert f"threshold on {1 if readable else 0})" in n.d.log()
    _set_state(n, "gpu0.badpages", 10)
    if readable:
        n.wait_health(lambda h: h[ids[0]] == "Unhealthy")
    else:
        time.sleep(0.5)
        assert "retired HBM pages" not in n.d.log()


def test_in_process_regeneration_is_an_event_gap(mk):
    """Without the relay, every monitor generation registers amdsmi events
    afresh: a GPU_POST_RESET sent between the old registration and the new one
    reached nobody. A GPU waiting for it across that gap goes back in service
    once amdsmi has answered every poll for --reset-recovery-hold-ms."""
    n = mk(args=["--reset-recovery-hold-ms", "1000"])
    ids = sorted(n.start())
    n.inject("0 3 pre-reset")
    n.wait_health(lambda h: h[ids[0]] == "Unhealthy")
    time.sleep(1.5)  # no gap yet: the hold does not run
    assert "recovered without GPU_POST_RESET" not in n.d.log()
    n.d.signal(signal.SIGHUP)
    assert n.first_law() == {ids[0]: "Unhealthy", ids[1]: "Healthy"}
    log = n.d.wait_log("waits for GPU_POST_RESET across an event gap")
    assert "registration renewed by a new monitor generation" in log
    n.wait_health(lambda h: h[ids[0]] == "Healthy", timeout=10)
    assert n.d.log().count("recovered without GPU_POST_RESET") == 1


def test_hold_zero_keeps_the_strict_rule(mk):
    """--reset-recovery-hold-ms=0: only the event brings the GPU back, gap or not."""
    n = mk(args=["--reset-recovery-hold-ms", "0"])
    ids = sorted(n.start())
    n.inject("0 3 pre-reset")
    n.wait_health(lambda h: h[ids[0]] == "Unhealthy")
    n.d.signal(signal.SIGHUP)
    assert n.first_law() == {ids[0]: "Unhealthy", ids[1]: "Healthy"}
    assert "only the event (or the operator) brings it back" in n.d.wait_log("across an event gap")
    time.sleep(1.0)
    assert "recovered without" not in n.d.log()
    n.inject("0 4 post-reset")
    n.wait_health(lambda h: h[ids[0]] == "Healthy")


def test_failing_event_waits_are_a_gap(mk):
    """In-process event waits that keep failing (ADP_EVENT_FAIL_MS) deliver no
    GPU_POST_RESET either: a GPU waiting across them is recovered by polling;
    a new GPU_PRE_RESET afterwards starts a fresh wait that only a new gap (or
    the event) ends."""
    n = mk(args=["--reset-recovery-hold-ms", "800"], env={"ADP_EVENT_FAIL_MS": "300"})
    ids = sorted(n.start())
    n.inject("1 3 pre-reset")
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    n.inject("fail 20")  # ~2 s of failed waits
    n.d.wait_log("amdsmi event waits have failed for")
    n.wait_health(lambda h: h[ids[1]] == "Healthy", timeout=10)
    assert "event gap (amdsmi event waits failing)" in n.d.log()
    n.d.wait_log("amdsmi event waits succeed again", timeout=10)
    n.inject("1 3 pre-reset again")
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    time.sleep(1.6)  # twice the hold: no gap since this PRE_RESET
    assert n.d.log().count("recovered without GPU_POST_RESET") == 1
    n.inject("1 4 post-reset")
    n.wait_health(lambda h: h[ids[1]] == "Healthy")


def _settled(d, timeout=30):
    """Waits until the daemon's last SIGHUP has been followed by a running
    health monitor (SIGHUPs sent while one is pending coalesce, so counting
    them does not work)."""
    deadline = time.monotonic() + timeout
    while True:
        log = d.log()
        if log.rfind("health monitor watching") > log.rfind("received SIGHUP"):
            return
        assert time.monotonic() < deadline, log[-3000:]
        time.sleep(0.05)


def test_in_process_sighup_storm_with_resets_leaves_no_gpu_stuck(mk):
    """SIGHUPs back to back with PRE/POST pairs injected around them, and every
    third POST_RESET dropped (as a real registration gap would lose it): every
    GPU ends Healthy -- by the event when it arrives, by the polled check
    across the gaps when it does not."""
    import random
    rnd = random.Random(11)
    n = mk(args=["--reset-recovery-hold-ms", "800", "--reset-flap-limit", "0"])  # (6 resets per GPU)
    ids = sorted(n.start())
    for i in range(12):
        gpu = i % 2
        if i % 3 == 2:
            # The reset whose POST is lost must be one seen before the gap: a
            # PRE_RESET written during a restart may be lost with the mock's
            # event FIFO (as real amdsmi loses it) or read after it.
            _settled(n.d)
            n.inject(f"{gpu} 3 storm pre {i}")
            n.d.wait_log(f"storm pre {i}", timeout=30)
        else:
            n.inject(f"{gpu} 3 storm pre {i}")
        n.d.signal(signal.SIGHUP)
        time.sleep(rnd.uniform(0, 0.2))
        if i % 3 != 2:  # 2, 5, 8, 11 lost -- the last one too
            n.inject(f"{gpu} 4 storm post {i}")
        time.sleep(rnd.uniform(0, 0.2))
    deadline = time.monotonic() + 30
    h = None
    while True:
        try:
            h = n.first_law(timeout=2)
        except Exception:
            pass
        if h == {ids[0]: "Healthy", ids[1]: "Healthy"}:
            break
        assert time.monotonic() < deadline, (h, n.d.log()[-3000:])
        try:
            h = n.wait_health(lambda x: x == {ids[0]: "Healthy", ids[1]: "Healthy"}, timeout=3)
            break
        except Exception:
            continue
    assert n.d.log().count("received SIGHUP") >= 4  # (signals sent while one is pending coalesce)
    assert "recovered without GPU_POST_RESET" in n.d.log()  # GPU 1's last reset: only polling ended it


def test_a_flapping_gpu_is_quarantined_until_a_quiet_window(mk):
    """--reset-flap-limit 3 within --reset-flap-window-ms: the third
    GPU_PRE_RESET in the window keeps the GPU out of service (cause
    "flapping"); its GPU_POST_RESET no longer brings it back, a SIGHUP does not
    either; once a whole window passes without a reset it is Healthy again. The
    other GPU is untouched, and two resets stay under the limit."""
    n = mk(args=["--reset-flap-limit", "3", "--reset-flap-window-ms", "2500", "--metrics-addr", "127.0.0.1:0"])
    ids = sorted(n.start())
    for i in range(2):
        n.inject(f"1 3 pre {i}")
        n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
        n.inject(f"1 4 post {i}")
        n.wait_health(lambda h: h[ids[1]] == "Healthy")
    n.inject("1 3 pre 2")
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    t_last = time.monotonic()
    assert "reset 3 times within 2 s: quarantined" in n.d.wait_log("quarantined")
    n.inject("1 4 post 2")
    n.d.wait_log("post 2")
    time.sleep(0.3)
    assert n.q.empty() or all(health(n.q.get_nowait())[ids[1]] == "Unhealthy" for _ in range(n.q.qsize()))
    port = int(__import__("re").search(r"on port (\d+)", n.d.log()).group(1))
    from test_metrics import _get, _parse, _value
    bdf1 = n.fx["gpus"][1]["bdf"]
    s = _parse(_get(port, "/metrics")[1])
    assert _value(s, "amdgpu_dp_gpu_failure", bdf=bdf1, cause="flapping") == 1
    assert _value(s, "amdgpu_dp_gpu_failure", bdf=bdf1, cause="reset_pending") == 0
    n.d.signal(signal.SIGHUP)  # the quarantine outlives a restart
    assert n.first_law() == {ids[0]: "Healthy", ids[1]: "Unhealthy"}
    n.wait_health(lambda h: h[ids[1]] == "Healthy", timeout=10)
    assert time.monotonic() - t_last >= 2.4
    assert "quarantine over" in n.d.log()


def test_the_reset_history_survives_a_container_restart(mk):
    """With --health-state-file the resets counted for flap damping are kept
    with the verdicts (wall clock): two resets, a plugin container restart,
    and the third reset within the window quarantines the GPU -- a restart
    neither resets the count nor ends a quarantine early."""
    import tempfile
    state = os.path.join(tempfile.mkdtemp(prefix="adp-flap-"), "health.state")

    def make():
        return mk(args=["--reset-flap-limit", "3", "--reset-flap-window-ms", "60000", "--health-state-file", state])
    n = make()
    ids = sorted(n.start())
    for i in range(2):
        n.inject(f"1 3 pre {i}")
        n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
        n.inject(f"1 4 post {i}")
        n.wait_health(lambda h: h[ids[1]] == "Healthy")
    line = [ln for ln in open(state).read().splitlines() if ln.startswith(n.fx["gpus"][1]["uuid"])][0]
    assert len(line.split("\t")[5].split("=")[1].split(",")) == 2, line
    assert n.close() == 0
    n = make()  # a new process, the same state file
    assert n.start() == {ids[0]: "Healthy", ids[1]: "Healthy"}
    n.inject("1 3 pre 2")
    assert "reset 3 times within 60 s: quarantined" in n.d.wait_log("quarantined")
    n.inject("1 4 post 2")
    n.d.wait_log("post 2")
    assert n.close() == 0
    n = make()  # and the quarantine itself outlives the next restart
    assert n.start() == {ids[0]: "Healthy", ids[1]: "Unhealthy"}
    time.sleep(0.5)
    assert "quarantine over" not in n.d.log()


@pytest.mark.parametrize("query,busy,ok", [("vram_used", "busy", "100"), ("activity", "in-reset", "7")])
def test_polled_recovery_waits_for_the_driver_to_report_the_devices_memory(mk, query, busy, ok):
    """The polled recovery after an event gap needs more than amdsmi's cached
    UUID: the driver must report the device's VRAM usage too -- it does not
    while a reset is under way. Here the mock's VRAM query fails after the gap:
    the GPU stays out until it answers, then comes back once the hold has
    passed from there. The same for the SMU's activity metrics (the driver
    refuses them while the GPU is in reset)."""
    n = mk(args=["--reset-recovery-hold-ms", "600"])
    ids = sorted(n.start())
    n.d.wait_log("health poll #1")  # VRAM usage read at least once
    n.inject("1 3 pre-reset")
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    vram = os.path.join(n.state, f"gpu1.{query}")
    with open(vram, "w") as f:
        f.write(busy + "\n")  # the driver does not answer about the device
    n.d.signal(signal.SIGHUP)  # an in-process registration gap
    assert n.first_law() == {ids[0]: "Healthy", ids[1]: "Unhealthy"}
    n.d.wait_log("across an event gap")
    time.sleep(1.5)  # more than twice the hold
    assert "recovered without GPU_POST_RESET" not in n.d.log()
    with open(vram, "w") as f:
        f.write(ok + "\n")
    t0 = time.monotonic()
    n.wait_health(lambda h: h[ids[1]] == "Healthy", timeout=10)
    assert time.monotonic() - t0 >= 0.5


def test_quarantine_and_operator_requests_apply_with_polling_off(mk, tmp_path):
    """DP_HEALTH_POLL_MS=0 turns liveness polling off, not the rest (round-5
    advice): a reset-flap quarantine still ends after a quiet window, and drains
    and return-to-service requests still apply, on the monitor's 1 s timer --
    before, all three ran only inside a poll, and a flapping GPU stayed out for
    good."""
    drain = str(tmp_path / "drain")
    n = mk(args=["--reset-flap-limit", "2", "--reset-flap-window-ms", "1500", "--drain-file", drain],
           env={"DP_HEALTH_POLL_MS": "0"})
    ids = sorted(n.start())
    assert "DP_HEALTH_POLL_MS=0: no liveness polls" in n.d.log()
    n.inject("1 3 pre 0")
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    n.inject("1 4 post 0")
    n.wait_health(lambda h: h[ids[1]] == "Healthy")
    n.inject("1 3 pre 1")
    n.wait_health(lambda h: h[ids[1]] == "Unhealthy")
    t_last = time.monotonic()
    n.inject("1 4 post 1")
    n.d.wait_log("quarantined")
    n.wait_health(lambda h: h[ids[1]] == "Healthy", timeout=8)  # no poll runs: the timer ended it
    assert time.monotonic() - t_last >= 1.4
    assert "quarantine over" in n.d.log()
    with open(drain, "w") as f:
        f.write(n.fx["gpus"][0]["bdf"] + "\n")
    n.wait_health(lambda h: h[ids[0]] == "Unhealthy", timeout=5)
    open(drain, "w").close()
    n.wait_health(lambda h: h[ids[0]] == "Healthy", timeout=5)
    n.inject("0 3 pre 2")  # a reset that never completes ...
    n.wait_health(lambda h: h[ids[0]] == "Unhealthy")
    with open(drain + ".return", "w") as f:  # ... and the operator's way back
        f.write(n.fx["gpus"][0]["bdf"] + "\n")
    n.wait_health(lambda h: h[ids[0]] == "Healthy", timeout=5)
    assert "returned to service by the operator" in n.d.log()

"""Events that name no known processor, opt-in extra event types, and the
rollback of a partial event registration (round-6 review items 1 and 3).

* Unmatched events. The reference makes every device Unhealthy when an event
  names no device (/root/reference/cmd/nvidia-device-plugin/nvidia.go:244-251).
  Here an event on a processor handle amdsmi never enumerated -- in-process,
  or one the event relay could not place ("node=- bdf=-") -- is logged as an
  ERROR and counted in amdgpu_dp_unmatched_events_total{type}; an unmatched
  GPU_PRE_RESET holds every GPU (reset pending, with a confirmed event gap, so
  the polled check brings each back after --reset-recovery-hold-ms). The mock
  delivers such events with FIFO lines "foreign <type>".
* --health-event-extra-types: KFD's informational events (PROCESS_START = 12,
  PROCESS_END = 13, ...) registered on top, counted per GPU and never a verdict.
* A registration that fails on one processor is undone on the ones before it
  (smi.cc EventsInit), and every stop releases whatever was registered: across
  SIGHUPs the mock's live registration count returns to what is expected and
  no handle is registered twice (reference nvidia.go:210-226 deletes its
  event set whatever happened).
"""

import os
import re
import signal
import subprocess
import time

import pytest

from k8s_gpu_sharing_plugin_amd import DAEMON, MOCK_LIB
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet, native

from test_event_relay import RelayNode
from test_health import Node
from test_metrics import _get, _parse


def _samples(port, name):
    m = _parse(_get(port, "/metrics")[1])
    return {tuple(sorted(ls)): v for (n, ls), v in m.items() if n == name}


def _wait_samples(port, name, want, timeout=5.0):
    deadline = time.monotonic() + timeout
    while True:
        got = _samples(port, name)
        if all(got.get(k) == v for k, v in want.items()) or time.monotonic() > deadline:
            return got
        time.sleep(0.05)


def _port(d):
    return int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))


def test_event_types_parse_and_classify():
    c = native.health_config("", "")
    assert all(c["verdicts"][str(t)] == 0 for t in range(5, 14)), c  # KFD's informational events: no verdict
    assert c["verdicts"]["3"] == -1 and c["verdicts"]["4"] == 1


@pytest.mark.parametrize("value", ["99", "0", "PROCESS_BEGIN", "12,x"])
def test_unknown_extra_event_type_is_refused(scratch, value):
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB,
               AMDSMI_MOCK_FIXTURE=fixtures.write(fixtures.node(1), scratch + ".fixture"))
    r = subprocess.run([DAEMON, "--device-plugin-path", scratch, "--health-event-extra-types", value],
                       capture_output=True, text=True, timeout=30, env=env)
    assert r.returncode == 1 and "invalid --health-event-extra-types option" in r.stdout + r.stderr, r


def test_extra_event_types_are_counted_never_a_verdict(scratch):
    n = Node(scratch, fixtures.node(2), args=["--metrics-addr", "127.0.0.1:0",
                                              "--health-event-extra-types", "12, process_end"])
    try:
        port = _port(n.d)
        bdf = [g["bdf"] for g in fixtures.node(2)["gpus"]]
        for line in ("0 12 4d2 python3", "0 13 4d2 python3", "1 12 4d3 probe", "1 5 migrate (not registered)"):
            n.inject(line)
        want = {(("bdf", bdf[0]), ("type", "PROCESS_START")): 1, (("bdf", bdf[0]), ("type", "PROCESS_END")): 1,
                (("bdf", bdf[1]), ("type", "PROCESS_START")): 1}
        got = _wait_samples(port, "amdgpu_dp_gpu_events_total", want)
        assert got == want, got  # MIGRATE_START (5) was not registered: the mock filters it, as amdsmi does
        time.sleep(0.3)
        assert n.q.empty()  # no health transition
        assert "events off" not in n.d.log()
    finally:
        n.close()


@pytest.mark.parametrize("layout", ["in-process", "relay"])
def test_unmatched_pre_reset_holds_every_gpu_until_polled_recovery(scratch, layout):
    hold = ["--reset-recovery-hold-ms", "600"]
    if layout == "relay":
        n = RelayNode(scratch, daemon_args=hold)
        d, relay = n.d, n.relay
        d.wait_log("events on through the relay")
        port = n.port
        health = n.health
    else:
        n = Node(scratch, fixtures.node(2), args=["--metrics-addr", "127.0.0.1:0", *hold],
                 env={"DP_HEALTH_POLL_MS": "100"})
        d, relay = n.d, None
        port = _port(d)

        def health(timeout=5):
            return [x.health for x in n.next(timeout).devices]
    try:
        n.inject("foreign 1 a VM fault on a handle nobody enumerated")
        n.inject("foreign 3 reset of a processor amdsmi never named")
        deadline = time.monotonic() + 10
        h = health()
        while h != ["Unhealthy", "Unhealthy"]:
            h = health(max(0.05, deadline - time.monotonic()))
        log = d.wait_log("GPU_PRE_RESET(3) on a processor that matches no GPU of this node")
        assert "every GPU is held until the polled check" in log
        got = _wait_samples(port, "amdgpu_dp_unmatched_events_total",
                            {(("type", "GPU_PRE_RESET"),): 1, (("type", "VMFAULT"),): 1})
        assert got == {(("type", "GPU_PRE_RESET"),): 1, (("type", "VMFAULT"),): 1}, got
        import subprocess
        import sys
        st = subprocess.run([sys.executable, "-m", "k8s_gpu_sharing_plugin_amd", "status",
                             f"http://127.0.0.1:{port}/metrics"], capture_output=True, text=True, timeout=60)
        assert "UNMATCHED events (amdsmi named a processor no GPU of this node is): GPU_PRE_RESET x1, VMFAULT x1" \
            in st.stdout, st.stdout
        if relay is not None:
            rlog = relay.wait_log("forwarded unplaced")
            assert "processor handle amdsmi did not enumerate" in rlog
            assert "the event relay could not place it either" in log
        else:
            assert "amdsmi named a processor handle it never enumerated" in log
        # back after the hold, by the polled check (no GPU_POST_RESET can be placed)
        deadline = time.monotonic() + 10
        while h != ["Healthy", "Healthy"]:
            h = health(max(0.05, deadline - time.monotonic()))
        rec = _samples(port, "amdgpu_dp_gpu_recovered_without_event_total")
        assert sorted(rec.values()) == [1, 1], rec
        assert d.log().count("recovered without GPU_POST_RESET") == 2
    finally:
        (n.stop if layout == "relay" else n.close)()


def test_unmatched_post_reset_and_ignored_types_change_nothing(scratch):
    n = Node(scratch, fixtures.node(2), args=["--metrics-addr", "127.0.0.1:0"])
    try:
        port = _port(n.d)
        for line in ("foreign 4 post", "foreign 2 thermal", "foreign 12 not registered anywhere"):
            n.inject(line)
        want = {(("type", "GPU_POST_RESET"),): 1, (("type", "THERMAL_THROTTLE"),): 1,
                (("type", "PROCESS_START"),): 1, (("type", "GPU_PRE_RESET"),): 0}
        got = _wait_samples(port, "amdgpu_dp_unmatched_events_total", want)
        assert got == want, got
        time.sleep(0.3)
        assert n.q.empty()
        assert n.d.log().count("matches no GPU of this node") == 3
    finally:
        n.close()


def test_relay_event_on_a_gpu_this_daemon_does_not_serve_is_not_unmatched(scratch):
    n = RelayNode(scratch, daemon_args=["--devices", "0"])
    try:
        n.d.wait_log("events on through the relay")
        n.inject("1 3 reset of the GPU another daemon serves")
        n.inject("0 1 fault here")  # in order after it: once this is seen, the other was handled
        n.d.wait_log("VMFAULT(1) on GPU 0")
        assert _samples(n.port, "amdgpu_dp_unmatched_events_total") == {(("type", "GPU_PRE_RESET"),): 0}
        time.sleep(0.2)
        assert n.q.empty()
    finally:
        n.stop()


def test_relay_event_on_a_processor_the_daemon_does_not_know_is_unmatched(scratch):
    """The relay places an event (KFD node, PCI address) on a GPU that is in no
    enumeration of the daemon's (here the relay sees a third GPU): the daemon
    cannot place it -- an ERROR and a counter, and a GPU_PRE_RESET holds every
    GPU it serves until the polled check, as for an unplaceable one."""
    n = RelayNode(scratch, relay_gpus=3, daemon_args=["--reset-recovery-hold-ms", "600"])
    try:
        n.d.wait_log("events on through the relay")
        third = fixtures.node(3)["gpus"][2]["bdf"]
        n.inject("2 3 reset of a GPU only the relay knows")
        deadline = time.monotonic() + 10
        h = n.health()
        while h != ["Unhealthy", "Unhealthy"]:
            h = n.health(max(0.05, deadline - time.monotonic()))
        log = n.d.wait_log("GPU_PRE_RESET(3) on a processor that matches no GPU of this node")
        assert "the relay's processor (node " in log and f"{third} partition 0) is none of this daemon's" in log
        assert _samples(n.port, "amdgpu_dp_unmatched_events_total") == {(("type", "GPU_PRE_RESET"),): 1}
        deadline = time.monotonic() + 10
        while h != ["Healthy", "Healthy"]:  # no GPU_POST_RESET can be placed: the polled check
            h = n.health(max(0.05, deadline - time.monotonic()))
    finally:
        n.stop()


@pytest.mark.parametrize("layout", ["in-process", "relay"])
def test_one_reset_of_a_partitioned_gpu_is_one_reset(scratch, layout):
    """KFD reports a GPU reset on every KFD node of the GPU: on a CPX MI355X
    that is 8 GPU_PRE_RESETs, then 8 GPU_POST_RESETs, for one reset. Counted
    per event, one reset quarantined the GPU for a whole flap window (found by
    the health model check once its I8 counted resets, not events). It is one
    reset: the GPU is back after its POST_RESETs, and it takes
    --reset-flap-limit such resets to quarantine it."""
    cpx = fixtures.node(2, modes="CPX")
    args = ["--partition-strategy", "single", "--reset-flap-limit", "2", "--metrics-addr", "127.0.0.1:0"]
    if layout == "relay":
        n = RelayNode(scratch, fx=cpx, daemon_args=args)
        n.d.wait_log("events on through the relay")
        q, stop = n.q, n.stop
    else:
        n = Node(scratch, cpx, args=args, env={"DP_HEALTH_POLL_MS": "100"})
        q, stop = n.q, n.close

    def unhealthy(timeout=5):
        return sum(d.health != "Healthy" for d in q.get(timeout=timeout).devices)
    try:
        for rnd in range(2):
            for p in range(8):
                n.inject(f"0:{p} 3 reset {rnd} pre on partition {p}")
            while unhealthy() != 8:
                pass
            for p in range(8):
                n.inject(f"0:{p} 4 reset {rnd} post on partition {p}")
            if rnd == 0:
                while unhealthy() != 0:  # one reset: back in service
                    pass
                assert "quarantined" not in n.d.log()
        # the second reset reaches --reset-flap-limit 2: its POST_RESETs do not bring it back
        assert "GPU 0000:0c:00.0 reset 2 times within" in n.d.wait_log("reset 2 times within")
        n.d.wait_log("reset 1 post on partition 7")
        time.sleep(0.3)
        last = None
        while not q.empty():
            last = q.get_nowait()
        assert last is None or sum(d.health != "Healthy" for d in last.devices) == 8
        assert _samples(n.port if layout == "relay" else _port(n.d), "amdgpu_dp_gpu_failure") \
            .get((("bdf", "0000:0c:00.0"), ("cause", "flapping"))) == 1
    finally:
        stop()


def _evt(path):
    text = open(path).read() if os.path.exists(path) else ""
    return {k: int(v) for k, v in re.findall(r"(\w+)=(\d+)", text)}


@pytest.mark.parametrize("fail_on", [None, [1]])
def test_event_registration_is_never_leaked_across_reloads(scratch, tmp_path, fail_on):
    """GPU 1's registration fails (fail_on=[1]): the one made on GPU 0 is undone,
    events are off (polling), and every SIGHUP generation starts from zero live
    registrations -- nothing registered twice, nothing left at shutdown. Without
    the fault, each generation holds exactly one registration per processor."""
    fx = fixtures.node(2)
    if fail_on:
        fx["evt_init_fail_on"] = fail_on
    evt = str(tmp_path / "evt")
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, env={"AMDSMI_MOCK_EVT_FILE": evt, "DP_HEALTH_POLL_MS": "100"}).start()
    try:
        k.wait_registration()
        d.wait_log("health monitor watching")
        want_live = 0 if fail_on else 2
        for gen in range(1, 5):
            if gen > 1:
                d.signal(signal.SIGHUP)
                d.wait_log("health monitor watching", count=gen, timeout=15)
            s = _evt(evt)
            assert s["live"] == want_live and s["double_init"] == 0 and s["leaked_at_shutdown"] == 0, (gen, s)
        log = d.log()
        if fail_on:
            assert log.count("undoing the 1 made before it") == 4, log[-3000:]
            assert "events off: amdsmi event notification unavailable" in log
    finally:
        assert d.stop() == 0
        k.stop()
    s = _evt(evt)
    assert s["live"] == 0 and s["double_init"] == 0 and s["leaked_at_shutdown"] == 0, s
    assert s["stops"] >= s["inits"], s


@pytest.mark.parametrize("fail_on", [None, [1]])
def test_event_probe_cycles_register_and_stop_everything(scratch, tmp_path, fail_on):
    """amdgpu-dp-event-probe --cycles N (what the GPU test runs on the real
    library): N generations of EventsInit + EventsStopAll, then the waiting
    registration. On the mock each generation holds one registration per
    processor and none after its stop; with GPU 1's init failing, none at all."""
    from k8s_gpu_sharing_plugin_amd import binary
    import json
    fx = fixtures.node(2)
    if fail_on:
        fx["evt_init_fail_on"] = fail_on
    evt = str(tmp_path / "evt")
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=fixtures.write(fx, scratch + ".fixture"),
               AMDSMI_MOCK_EVT_FILE=evt)
    r = subprocess.run([binary("amdgpu-dp-event-probe"), "--lib", MOCK_LIB, "--cycles", "3", "--wait-ms", "300"],
                       capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(rec["cycles"]) == 3, rec
    for c in rec["cycles"]:
        assert c["after_stop"] == 0, rec
        if fail_on:
            assert c["init"] != "ok" and c["registered"] == 0, rec
        else:
            assert c["init"] == "ok" and c["registered"] == 2, rec
    assert (rec["registration"] == "ok") == (not fail_on), rec
    assert rec["cycle_count"] == 3 and rec["cycles_ok"] == (0 if fail_on else 3), rec
    assert rec["fds_after_cycles"] == rec["fds_after_first_cycle"] == rec["fds_before_cycles"], rec
    s = _evt(evt)
    assert s["live"] == 0 and s["double_init"] == 0 and s["leaked_at_shutdown"] == 0, s


def test_relay_never_leaks_a_registration_across_renewals(scratch, tmp_path):
    """The relay's renewals (a daemon with a different processor view, or
    events off) stop whatever the last one registered, complete or not."""
    fx = dict(fixtures.node(2), evt_init_fail_on=[1])
    evt = str(tmp_path / "evt")
    sock = os.path.join(scratch + ".fixture", "events.sock")
    os.makedirs(scratch + ".fixture", exist_ok=True)
    rdir = scratch + "-relay"
    os.makedirs(rdir, exist_ok=True)
    relay = harness.Daemon(rdir, fx, args=["--event-relay", "--health-event-socket", sock],
                           env={"AMDSMI_MOCK_EVT_FILE": evt}).start()
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = None
    try:
        relay.wait_log("event notification unavailable")
        d = harness.Daemon(scratch, fx, args=["--health-event-socket", sock],
                           env={"DP_HEALTH_POLL_MS": "100"}).start()
        k.wait_registration()
        for gen in range(1, 4):
            if gen > 1:
                d.signal(signal.SIGHUP)
            relay.wait_log("re-enumerating (a daemon asked: events are off)", count=gen, timeout=15)
            relay.wait_log("event notification unavailable", count=gen + 1, timeout=15)
            s = _evt(evt)
            assert s["live"] == 0 and s["double_init"] == 0 and s["leaked_at_shutdown"] == 0, (gen, s)
    finally:
        if d:
            d.stop()
        k.stop()
        assert relay.stop() == 0
    s = _evt(evt)
    assert s["live"] == 0 and s["double_init"] == 0 and s["leaked_at_shutdown"] == 0, s


def test_hosted_monitor_and_relay_on_the_mock(scratch, tmp_path):
    """The C API's hosted monitor and relay (what the GPU tests run next to HIP,
    utils/hosted_events.py) on the mock: an event reaches the hosted monitor's
    counters, and the hosted relay forwards one to a real daemon."""
    fifo = str(tmp_path / "events")
    os.mkfifo(fifo)
    fx = dict(fixtures.node(2), event_fifo=fifo)
    fxpath = fixtures.write(fx, scratch + ".fixture")
    old = {k: os.environ.get(k) for k in ("AMD_SMI_LIB", "AMDSMI_MOCK_FIXTURE")}
    os.environ["AMD_SMI_LIB"], os.environ["AMDSMI_MOCK_FIXTURE"] = MOCK_LIB, fxpath
    try:
        m = native.HostedMonitor(extra_types="12,13", devices=(0, 1))
        try:
            fd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
            os.write(fd, b"1 12 4d2 python3\n")
            os.close(fd)
            deadline = time.monotonic() + 5
            st = m.state()
            while not st["events"] and time.monotonic() < deadline:
                time.sleep(0.05)
                st = m.state()
            assert st["events"] == [{"bdf": fx["gpus"][1]["bdf"], "type": "PROCESS_START", "n": 1}], st
            assert st["events_enabled"] == 1 and st["registrations"] == 2 and st["transitions"] == [], st
        finally:
            m.close()
        sock = str(tmp_path / "relay.sock")
        r = native.HostedRelay(sock, extra_types="12")
        k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        d = harness.Daemon(scratch, fx, args=["--health-event-socket", sock, "--metrics-addr", "127.0.0.1:0"]).start()
        try:
            port = _port(d)
            d.wait_log("events on through the relay")
            fd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
            os.write(fd, b"0 12 4d3 probe\n")
            os.close(fd)
            want = {(("bdf", fx["gpus"][0]["bdf"]), ("type", "PROCESS_START")): 1}
            assert _wait_samples(port, "amdgpu_dp_gpu_events_total", want) == want
        finally:
            d.stop()
            k.stop()
            assert r.close() == 0
    finally:
        for key, v in old.items():
            if v is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = v

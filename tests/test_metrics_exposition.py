"""/metrics through a real Prometheus exposition parser, in every layout.

prometheus_client's own parser (text_string_to_metric_families) reads the
scrape of each deployment layout -- plain; events through the relay; memory
units enforced with per-grant accounting and the driver-side scan; the kubelet
PodResources link -- and the checks are what a Prometheus server would reject
or silently mangle: one HELP and one TYPE per family, every sample inside a
declared family, no duplicate series, and label values from outside
(pod, namespace and container names with quotes, backslashes and newlines)
escaped so they read back exactly.

Parity: the reference exports no metrics; the daemon families are
native/src/daemon/daemon_metrics.cc, the plugin families plugin_metrics.cc.
"""

import os
import re
import time

import pytest

from k8s_gpu_sharing_plugin_amd import BUILD_DIR
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

from test_metrics import PodResourcesStub, _get, _list_response, _preloadable_shim, _wait_file

parser = pytest.importorskip("prometheus_client.parser")

SIM = os.path.join(BUILD_DIR, "libadp_devcgroup_sim.so")
HOSTILE = [('ml"ns\\', 'evil"pod\\name\nline2', 'c"{x}'), ("web", "infer,a=b", "srv\\")]


def check_exposition(text):
    """Parses a scrape; returns {family name: family}. Fails on anything a
    Prometheus server would refuse or misread."""
    lines = text.splitlines()
    helps = [ln.split()[2] for ln in lines if ln.startswith("# HELP ")]
    types = [ln.split()[2] for ln in lines if ln.startswith("# TYPE ")]
    assert len(helps) == len(set(helps)), sorted(h for h in helps if helps.count(h) > 1)
    assert len(types) == len(set(types)), sorted(t for t in types if types.count(t) > 1)
    assert set(helps) == set(types)
    # every sample line follows its own family's TYPE line
    declared, current = set(), None
    for ln in lines:
        if ln.startswith("# TYPE "):
            current = ln.split()[2]
            declared.add(current)
        elif ln and not ln.startswith("#"):
            name = re.match(r"[a-zA-Z_:][a-zA-Z0-9_:]*", ln).group(0)
            base = re.sub(r"_(bucket|sum|count)$", "", name)
            assert name == current or base == current, (ln, current)
    families = {f.name: f for f in parser.text_string_to_metric_families(text)}
    assert all(f.type != "unknown" for f in families.values()), [f.name for f in families.values()
                                                                 if f.type == "unknown"]
    seen = set()
    for f in families.values():
        for s in f.samples:
            key = (s.name, tuple(sorted(s.labels.items())))
            assert key not in seen, key
            seen.add(key)
    return families


def _samples(families, name):
    for f in families.values():
        for s in f.samples:
            if s.name == name:
                yield s


def _port(d):
    return int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))


def test_plain_layout(scratch):
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=["--metrics-addr", "127.0.0.1:0", "--pod-resources-socket",
                                                        ""]).start()
    try:
        port = _port(d)
        k.wait_registration()
        d.wait_log("health poll #1")
        fams = check_exposition(_get(port, "/metrics")[1])
        assert "amdgpu_dp_gpu_failure" in fams and "amdgpu_dp_allocatable" in fams
        assert "amdgpu_dp_pod_resources_up" not in fams  # no PodResources socket, no such series
        # counters keep their _total sample names
        assert {s.name for s in _samples(fams, "amdgpu_dp_restarts_total")} == {"amdgpu_dp_restarts_total"}
    finally:
        d.stop()
        k.stop()


def test_pod_resources_layout_escapes_hostile_names(scratch):
    pr_sock = os.path.join(scratch + ".fixture", "pod-resources.sock")
    os.makedirs(os.path.dirname(pr_sock), exist_ok=True)
    pr = PodResourcesStub(pr_sock)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=["--metrics-addr", "127.0.0.1:0", "--resource-config",
                                                        "gpu:sharedgpu:4", "--pod-resources-socket", pr_sock]).start()
    try:
        port = _port(d)
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        c.close()
        (ns0, pod0, c0), (ns1, pod1, c1) = HOSTILE
        pr.payload = _list_response([(ns0, pod0, c0, "amd.com/sharedgpu", ids[:2]),
                                     (ns1, pod1, c1, "amd.com/sharedgpu", [ids[4], "gone-replica-9"])])
        fams = check_exposition(_get(port, "/metrics")[1])
        ctr = {(s.labels["namespace"], s.labels["pod"], s.labels["container"]): s.value
               for s in _samples(fams, "amdgpu_dp_container_device_ids")}
        assert ctr == {(ns0, pod0, c0): 2, (ns1, pod1, c1): 1}  # read back exactly
        stale = [s.value for s in _samples(fams, "amdgpu_dp_stale_allocated_ids")]
        assert stale == [1]
    finally:
        pr.stop()
        d.stop()
        k.stop()


def test_relay_enforced_grants_and_driver_scan_layout(scratch, tmp_path):
    """The chart's layout with memory units enforced: events and driver-side
    scans through the relay, per-grant accounting files, PodResources with
    hostile names, a relayed event and a recovery counter per GPU."""
    shim, _check = _preloadable_shim()
    fifo = os.path.join(scratch + ".fixture", "events")
    os.makedirs(os.path.dirname(fifo), exist_ok=True)
    os.mkfifo(fifo)
    sock = os.path.join(scratch + ".fixture", "events.sock")
    fx = dict(fixtures.node(2), events_open_kfd=True)
    proc = tmp_path / "proc"
    proc.mkdir()
    relay = harness.Daemon(scratch + "-relay", fx, args=["--event-relay", "--health-event-socket", sock,
                                                         "--host-proc", str(proc)], event_fifo=fifo).start()
    relay.wait_log("relaying amdsmi events on")
    pr_sock = os.path.join(scratch + ".fixture", "pod-resources.sock")
    pr = PodResourcesStub(pr_sock)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    preload = " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), SIM) if x)
    d = harness.Daemon(scratch, fx, args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units",
        "--memcap-lib", shim, "--pod-resources-socket", pr_sock, "--health-event-socket", sock,
        "--driver-hbm-poll-ms", "100"], env={"LD_PRELOAD": preload, "DP_HEALTH_POLL_MS": "100"}).start()
    try:
        port = _port(d)
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        resp = c.allocate(ids[:3]).container_responses[0]
        c.close()
        host = [m for m in resp.mounts if m.container_path == "/run/amdgpu-dp/memcap"][0].host_path
        assert _wait_file(host)
        d.wait_log("events on through the relay")
        fd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
        os.write(fd, b"0 2 throttled\n")  # THERMAL_THROTTLE: counted, ignored
        os.close(fd)
        d.wait_log("THERMAL_THROTTLE(2) on GPU 0")
        (ns0, pod0, c0), _ = HOSTILE
        pr.payload = _list_response([(ns0, pod0, c0, "amd.com/gpu-mem-gb", ids[:3])])
        deadline = time.time() + 10
        while True:
            fams = check_exposition(_get(port, "/metrics")[1])
            if any(True for _ in _samples(fams, "amdgpu_dp_container_hbm_granted_bytes")) and \
                    any(s.value > 0 for s in _samples(fams, "amdgpu_dp_driver_hbm_polls_total")):
                break
            assert time.time() < deadline
            time.sleep(0.2)
        granted = [s for s in _samples(fams, "amdgpu_dp_container_hbm_granted_bytes")]
        assert [(s.labels["namespace"], s.labels["pod"], s.labels["container"]) for s in granted] == [(ns0, pod0, c0)]
        assert [s.value for s in _samples(fams, "amdgpu_dp_health_events_enabled")] == [1]
        ev = [s for s in _samples(fams, "amdgpu_dp_gpu_events_total")]
        assert [s.labels["type"] for s in ev] == ["THERMAL_THROTTLE"] and ev[0].value == 1
        rec = [s for s in _samples(fams, "amdgpu_dp_gpu_recovered_without_event_total")]
        assert len(rec) == 2 and all(s.value == 0 for s in rec)
        assert {s.labels["kind"] for s in _samples(fams, "amdgpu_dp_memory_unit_mib")} == {"mib"}
        assert [s.labels["source"] for s in _samples(fams, "amdgpu_dp_driver_hbm_scan_processes")] == ["proc"]
    finally:
        pr.stop()
        d.stop()
        k.stop()
        relay.stop()


def test_exposition_checker_catches_what_prometheus_rejects():
    """The checks above are not vacuous."""
    ok = "# HELP a_total x\n# TYPE a_total counter\na_total 1\n"
    check_exposition(ok)
    for bad in (ok + ok,                                                        # family twice
                ok + "a_total 2\n",                                             # duplicate series
                "# HELP b x\n# TYPE b gauge\nc 1\n",                            # sample outside its family
                "# HELP b x\n# TYPE b gauge\nb{l=\"a\"} 1\nb{l=\"a\"} 2\n"):
        with pytest.raises(AssertionError):
            check_exposition(bad)
    with pytest.raises(Exception):
        check_exposition('# HELP b x\n# TYPE b gauge\nb{l="a"b"} 1\n')  # unescaped quote


def test_daemon_binary_has_no_inline_exposition():
    """The supervisor hands its numbers to daemon_metrics.cc: no family is
    spelled out in supervisor.cc any more (round 4's 185-line lambda)."""
    src = open(os.path.join(os.path.dirname(__file__), "..", "native", "src", "daemon", "supervisor.cc")).read()
    assert "# HELP" not in src and "# TYPE" not in src
    body = src.split("int RunDaemon(", 1)[1]
    assert body.count("\n") < 120, body.count("\n")

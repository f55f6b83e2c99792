"""Prometheus /metrics and /healthz endpoint (--metrics-addr).

The reference has no metrics ("Metrics / logging / observability:
minimal"); this pins the endpoint the DaemonSet's scrape config and liveness
probe use: device/allocatable/health gauges per resource, per-RPC counters and
handler-time histograms, restart counter, and /healthz tracking plugin state.
"""

import os
import re
import time
import urllib.error
import urllib.request

import pytest

from k8s_gpu_sharing_plugin_amd import REPO_ROOT as ROOT
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet


def _get(port, path):
    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=5) as r:
            return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


def _parse(text):
    """{(name, frozenset(labels)): value} for every sample line."""
    out = {}
    for line in text.splitlines():
        if not line or line.startswith("#"):
            continue
        m = re.match(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(?:\{(.*)\})? (\S+)$', line)
        assert m, f"bad sample line: {line!r}"
        labels = frozenset(re.findall(r'(\w+)="((?:[^"\\]|\\.)*)"', m.group(2) or ""))
        out[(m.group(1), labels)] = float(m.group(3))
    return out


def _value(samples, name, **labels):
    want = set(labels.items())
    hits = [v for (n, ls), v in samples.items() if n == name and want <= set(ls)]
    assert len(hits) == 1, (name, labels, hits)
    return hits[0]


@pytest.fixture
def served(scratch):
    fx = fixtures.node(2)
    fifo = os.path.join(scratch + ".fixture", "events")
    os.makedirs(os.path.dirname(fifo), exist_ok=True)
    os.mkfifo(fifo)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, args=["--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:sharedgpu:3"],
                       event_fifo=fifo).start()
    text = d.wait_log("serving /metrics and /healthz on port")
    port = int(re.search(r"serving /metrics and /healthz on port (\d+)", text).group(1))
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    yield d, k, c, port, fifo
    c.close()
    d.stop()
    k.stop()


def test_metrics_exposition(served):
    d, k, c, port, _ = served
    q, call = c.watch()
    law = q.get(timeout=5)
    ids = [x.ID for x in law.devices]
    for _ in range(5):
        c.allocate([ids[0]])
    c.preferred(ids, size=2)
    status, text = _get(port, "/metrics")
    assert status == 200
    # Families are grouped: every TYPE line names a family not seen before.
    types = [l.split()[2] for l in text.splitlines() if l.startswith("# TYPE")]
    assert len(types) == len(set(types))
    s = _parse(text)
    r = "amd.com/sharedgpu"
    assert _value(s, "amdgpu_dp_devices", resource=r) == 2
    assert _value(s, "amdgpu_dp_allocatable", resource=r) == 6
    assert _value(s, "amdgpu_dp_healthy_devices", resource=r) == 2
    assert _value(s, "amdgpu_dp_registered", resource=r) == 1
    assert _value(s, "amdgpu_dp_rpc_total", resource=r, method="Allocate") == 5
    assert _value(s, "amdgpu_dp_rpc_total", resource=r, method="GetPreferredAllocation") == 1
    assert _value(s, "amdgpu_dp_handler_seconds_count", resource=r, method="Allocate") == 5
    assert _value(s, "amdgpu_dp_handler_seconds_bucket", resource=r, method="Allocate", le="+Inf") == 5
    assert _value(s, "amdgpu_dp_handler_seconds_sum", resource=r, method="Allocate") < 0.01
    # read -> reply residency of the 6 unary calls (one sample per batch answered together)
    n = _value(s, "amdgpu_dp_rpc_residency_seconds_count", resource=r)
    assert 1 <= n <= 6
    assert _value(s, "amdgpu_dp_rpc_residency_seconds_bucket", resource=r, le="+Inf") == n
    les = sorted(((float(dict(ls)["le"]), v) for (m, ls), v in s.items()
                  if m == "amdgpu_dp_rpc_residency_seconds_bucket" and dict(ls)["le"] != "+Inf"))
    assert len(les) == 7 and all(a[1] <= b[1] for a, b in zip(les, les[1:]))
    assert _value(s, "amdgpu_dp_rpc_residency_seconds_sum", resource=r) < 0.1
    assert _value(s, "amdgpu_dp_restarts_total") == 1
    assert _value(s, "amdgpu_dp_build_info") == 1
    assert _value(s, "amdgpu_dp_grpc_connections_total", resource=r) >= 2
    per_dev = [v for (n, ls), v in s.items() if n == "amdgpu_dp_device_healthy"]
    assert per_dev == [1.0, 1.0]
    call.cancel()


def test_metrics_follow_health_and_healthz(served):
    d, k, c, port, fifo = served
    # Registration reaches the kubelet before the daemon marks itself serving and
    # starts the health monitor (which opens the event FIFO): wait for both.
    d.wait_log("health monitor watching")
    deadline = time.time() + 5
    while time.time() < deadline and _get(port, "/healthz")[0] != 200:
        time.sleep(0.05)
    assert _get(port, "/healthz") == (200, "ok\n")
    fd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
    os.write(fd, b"1 3 pre-reset\n")
    os.close(fd)
    deadline = time.time() + 5
    while time.time() < deadline:
        s = _parse(_get(port, "/metrics")[1])
        if _value(s, "amdgpu_dp_healthy_devices", resource="amd.com/sharedgpu") == 1:
            break
        time.sleep(0.05)
    assert _value(s, "amdgpu_dp_healthy_devices", resource="amd.com/sharedgpu") == 1
    assert sorted(v for (n, ls), v in s.items() if n == "amdgpu_dp_device_healthy") == [0.0, 1.0]
    assert _get(port, "/nope")[0] == 404
    # kubelet goes away and comes back: restart counter moves, healthz stays up after re-registration
    k.stop()
    k2 = kubelet.StubKubelet(k.socket_path).start()
    k2.wait_registration()
    deadline = time.time() + 5
    while time.time() < deadline and _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_restarts_total") < 2:
        time.sleep(0.05)
    assert _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_restarts_total") == 2
    # (as at start: Register() reaches the kubelet just before the plugin marks
    # itself serving again)
    deadline = time.time() + 5
    while time.time() < deadline and _get(port, "/healthz")[0] != 200:
        time.sleep(0.05)
    assert _get(port, "/healthz")[0] == 200
    k2.stop()


def test_slow_clients_do_not_hold_up_healthz(served):
    """Idle / trickling HTTP clients each have their own 2 s budget and are
    served side by side: the liveness probe on /healthz answers at once, and a
    client that never finishes its request is closed at its deadline."""
    import socket
    _, _, _, port, _ = served
    idle = []
    for _ in range(20):
        s = socket.create_connection(("127.0.0.1", port))
        s.sendall(b"GET /metr")  # never finishes the request line
        idle.append(s)
    t = time.time()
    assert _get(port, "/healthz")[0] in (200, 503)
    assert _get(port, "/metrics")[0] == 200
    assert time.time() - t < 1.0
    idle[0].settimeout(4)
    assert idle[0].recv(100) == b""  # closed by the server after its 2 s
    for s in idle:
        s.close()


def test_metrics_addr_invalid(scratch):
    d = harness.Daemon(scratch, args=["--metrics-addr", "nohost:notaport"]).start()
    assert d.proc.wait(10) == 1
    assert "invalid --metrics-addr" in d.log()


def test_builtin_sampler_writes_profile(scratch):
    """ADP_PROFILE_OUT: the daemon's own CPU sampler reports where its time went."""
    out = os.path.join(scratch + ".fixture", "profile.txt")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, env={"ADP_PROFILE_OUT": out, "ADP_PROFILE_HZ": "2000"}).start()
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    deadline = time.time() + 1.0
    while time.time() < deadline:
        c.allocate([ids[0]])
    c.close()
    assert d.stop() == 0
    k.stop()
    text = open(out).read()
    assert text.startswith("samples ")
    assert "== by shared object ==" in text and "== by symbol ==" in text


def _preloadable_shim():
    """The HBM-cap shim and its check program from BUILD_DIR, or a skip when
    that is a sanitizer build (the shim then needs its runtime preloaded first:
    the e2e sanitizer suites run the daemon, not workloads)."""
    import subprocess
    from k8s_gpu_sharing_plugin_amd import BUILD_DIR
    shim = os.path.join(BUILD_DIR, "libadp_memcap.so")
    deps = subprocess.run(["ldd", shim], capture_output=True, text=True).stdout
    if "libasan" in deps or "libtsan" in deps:
        pytest.skip("sanitizer build of the shim")
    return shim, os.path.join(BUILD_DIR, "adp_memcap_check")


def _wait_file(path, timeout=5.0):
    """Grant files are written by the daemon's background writer, just after
    Allocate() returns (long before a runtime would mount them)."""
    deadline = time.time() + timeout
    while not os.path.isfile(path) and time.time() < deadline:
        time.sleep(0.005)
    return os.path.isfile(path)


# --- kubelet PodResources: who holds which device -------------------------------

def _pb_len(field, payload: bytes) -> bytes:
    def varint(v):
        out = b""
        while v >= 0x80:
            out += bytes([(v & 0x7F) | 0x80])
            v >>= 7
        return out + bytes([v])
    return varint(field << 3 | 2) + varint(len(payload)) + payload


def _list_response(pods):
    """pods: [(namespace, pod, container, resource, [ids])] -> ListPodResourcesResponse bytes."""
    out = b""
    for ns, pod, ctr, res, ids in pods:
        devs = _pb_len(1, res.encode()) + b"".join(_pb_len(2, i.encode()) for i in ids)
        container = _pb_len(1, ctr.encode()) + _pb_len(2, devs)
        out += _pb_len(1, _pb_len(1, pod.encode()) + _pb_len(2, ns.encode()) + _pb_len(3, container))
    return out


class PodResourcesStub:
    def __init__(self, path):
        import grpc
        from concurrent import futures
        self.payload = b""
        self.calls = 0

        def handle(req, ctx):
            self.calls += 1
            return self.payload
        h = grpc.method_handlers_generic_handler(
            "v1.PodResourcesLister", {"List": grpc.unary_unary_rpc_method_handler(handle)})
        self.server = grpc.server(futures.ThreadPoolExecutor(2), handlers=[h])
        self.server.add_insecure_port("unix:" + path)
        self.server.start()

    def stop(self):
        self.server.stop(0)



def test_pod_resources_answer_over_the_bound_fails_the_call(scratch):
    """A PodResources answer past 16 MiB (the kubelet's own client's bound) is
    not held: the call fails, the scrape still answers, and the next good
    answer is used. (native/src/grpc/client.cc kMaxRecvBytes.)"""
    pr_sock = os.path.join(scratch + ".fixture", "pod-resources.sock")
    os.makedirs(os.path.dirname(pr_sock), exist_ok=True)
    pr = PodResourcesStub(pr_sock)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:sharedgpu:4",
        "--pod-resources-socket", pr_sock]).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        c.close()
        pr.payload = _list_response([("ml", "huge", "main", "amd.com/sharedgpu", [ids[0], "x" * (17 << 20)])])
        t0 = time.time()
        s = _parse(_get(port, "/metrics")[1])
        assert time.time() - t0 < 1.9
        assert _value(s, "amdgpu_dp_pod_resources_up") == 0
        assert pr.calls == 1
        pr.payload = _list_response([("ml", "train-a", "main", "amd.com/sharedgpu", [ids[0]])])
        s = _parse(_get(port, "/metrics")[1])
        assert _value(s, "amdgpu_dp_pod_resources_up") == 1
        assert _value(s, "amdgpu_dp_container_device_ids", device=ids[0].split("-replica-")[0], namespace="ml",
                      pod="train-a") == 1
        assert d.proc.poll() is None
    finally:
        pr.stop()
        d.stop()
        k.stop()

def test_pod_resources_sharing_metrics(scratch):
    pr_sock = os.path.join(scratch + ".fixture", "pod-resources.sock")
    os.makedirs(os.path.dirname(pr_sock), exist_ok=True)
    pr = PodResourcesStub(pr_sock)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:sharedgpu:4",
        "--pod-resources-socket", pr_sock]).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        c.close()
        g0 = ids[0].split("-replica-")[0]
        g1 = ids[4].split("-replica-")[0]
        pr.payload = _list_response([
            ("ml", "train-a", "main", "amd.com/sharedgpu", [ids[0], ids[1]]),
            ("ml", "train-b", "main", "amd.com/sharedgpu", [ids[2]]),
            ("web", "infer", "srv", "amd.com/sharedgpu", [ids[4]]),
            ("other", "cpu-pod", "x", "example.com/foo", ["whatever"]),
        ])
        s = _parse(_get(port, "/metrics")[1])
        r = "amd.com/sharedgpu"
        assert _value(s, "amdgpu_dp_pod_resources_up") == 1
        assert _value(s, "amdgpu_dp_device_allocated_ids", resource=r, device=g0) == 3
        assert _value(s, "amdgpu_dp_device_pods", resource=r, device=g0) == 2
        assert _value(s, "amdgpu_dp_device_pods", resource=r, device=g1) == 1
        assert _value(s, "amdgpu_dp_container_device_ids", device=g0, namespace="ml", pod="train-a") == 2
        _get(port, "/metrics")
        assert pr.calls == 1  # cached between scrapes
        pr.stop()
        pr = None
        time.sleep(2.1)
        s = _parse(_get(port, "/metrics")[1])
        assert _value(s, "amdgpu_dp_pod_resources_up") == 0
        assert not any(n == "amdgpu_dp_device_pods" for (n, _) in s)
    finally:
        if pr:
            pr.stop()
        d.stop()
        k.stop()


def test_health_liveness_is_reported(scratch):
    """Events registered or not (and why), polls, ECC reads: in the log after the
    first poll, in /metrics and in the SIGUSR1 dump (the real-GPU test asserts
    on the same report)."""
    import signal
    state = os.path.join(scratch + ".fixture", "state")
    os.makedirs(state, exist_ok=True)
    fx = fixtures.node(2)
    fx["events_supported"] = False
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, args=["--metrics-addr", "127.0.0.1:0"], state_dir=state,
                       env={"DP_HEALTH_POLL_MS": "100"}).start()
    try:
        text = d.wait_log("serving /metrics and /healthz on port")
        port = int(re.search(r"serving /metrics and /healthz on port (\d+)", text).group(1))
        k.wait_registration()
        log = d.wait_log("health poll #1:")
        assert re.search(r"health poll #1: 2/2 GPU\(s\) responding, uncorrectable ECC readable on 2 "
                         r"\(counts \[0,0\]\), retired pages readable on 2 \(threshold on 0\); events off: ",
                         log), log
        with open(os.path.join(state, "gpu1.badpages"), "w") as f:
            f.write("3\n")
        with open(os.path.join(state, "gpu0.vram_used"), "w") as f:
            f.write("1234\n")
        time.sleep(0.35)
        s = _parse(_get(port, "/metrics")[1])
        assert sorted(v for (n, ls), v in s.items() if n == "amdgpu_dp_retired_pages") == [0.0, 3.0]
        assert sorted(v for (n, ls), v in s.items() if n == "amdgpu_dp_gpu_hbm_used_bytes") == [0.0, 1234 << 20]
        assert sorted(v for (n, ls), v in s.items() if n == "amdgpu_dp_gpu_hbm_total_bytes") == \
            [float(fixtures.MI355X_VRAM_MIB << 20)] * 2
        assert _value(s, "amdgpu_dp_health_retired_page_reads_total", result="ok") >= 4
        assert _value(s, "amdgpu_dp_health_events_enabled") == 0
        assert _value(s, "amdgpu_dp_health_polls_total") >= 2
        assert _value(s, "amdgpu_dp_health_ecc_reads_total", result="ok") >= 4
        assert _value(s, "amdgpu_dp_health_ecc_reads_total", result="error") == 0
        d.signal(signal.SIGUSR1)
        d.wait_log('health: {"events": "off", "polls": ')
    finally:
        d.stop()
        k.stop()


def test_container_hbm_use_of_enforced_grants(scratch):
    """--enforce-memory-units with /metrics: each memory-unit container gets its
    grant's accounting file mounted (ADP_MEMCAP_FILE); the shim's processes
    count into it and /metrics reports used / granted / peak bytes and refused
    allocations per (pod, container, device). Files of containers the kubelet
    no longer lists are removed after two minutes."""
    import json
    import subprocess
    shim, check = _preloadable_shim()
    pr_sock = os.path.join(scratch + ".fixture", "pod-resources.sock")
    os.makedirs(os.path.dirname(pr_sock), exist_ok=True)
    pr = PodResourcesStub(pr_sock)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack",
        "--enforce-memory-units", "--memcap-lib", shim, "--pod-resources-socket", pr_sock]).start()
    holder = None
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        resp = c.allocate(ids[:3]).container_responses[0]
        c.close()
        envs = dict(resp.envs)
        assert envs["ADP_MEMCAP_FILE"] == "/run/amdgpu-dp/memcap"
        usage = [m for m in resp.mounts if m.container_path == "/run/amdgpu-dp/memcap"]
        assert len(usage) == 1 and not usage[0].read_only
        host = usage[0].host_path
        assert os.path.dirname(host) == os.path.join(scratch, "amdgpu-dp", "usage") and _wait_file(host)
        assert oct(os.stat(host).st_mode & 0o777) == "0o666"  # any uid in the container

        # The container: the shim (device 0 capped at 3000 MiB) with the file at its host path.
        env = dict(os.environ, LD_PRELOAD=" ".join(x for x in (os.environ.get("LD_PRELOAD", ""), shim) if x),
                   AMD_GPU_MEMORY_LIMIT_MIB=envs["AMD_GPU_MEMORY_LIMIT_MIB"], ADP_MEMCAP_FILE=host)
        env.pop("ADP_MEMCAP_KEY", None)
        holder = subprocess.Popen([check, "hold", "0", "2000"], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                  stderr=subprocess.DEVNULL, text=True, env=env)
        assert json.loads(holder.stdout.readline()) == {"step": "hold", "rc": 0}
        holder.stdout.readline()
        r = subprocess.run([check, "try", "0", "1500"], capture_output=True, text=True, timeout=30, env=env)
        assert json.loads(r.stdout.splitlines()[0])["rc"] == 2  # 2000 of 3000 held by the other process

        g0 = ids[0].split("-replica-")[0]
        pr.payload = _list_response([("ml", "infer", "srv", "amd.com/gpu-mem-gb", ids[:3])])
        s = _parse(_get(port, "/metrics")[1])
        lab = dict(namespace="ml", pod="infer", container="srv", device=g0)
        mib = 1 << 20
        assert _value(s, "amdgpu_dp_container_hbm_used_bytes", **lab) == 2000 * mib
        assert _value(s, "amdgpu_dp_container_hbm_granted_bytes", **lab) == 3000 * mib
        assert _value(s, "amdgpu_dp_container_hbm_peak_bytes", **lab) == 2000 * mib
        assert _value(s, "amdgpu_dp_container_hbm_refusals_total", **lab) == 1
        assert _value(s, "amdgpu_dp_container_hbm_processes", namespace="ml", pod="infer") == 1  # the holder
        holder.stdin.close()
        assert holder.wait(10) == 0
        holder = None
        time.sleep(2.1)  # PodResources cache
        s = _parse(_get(port, "/metrics")[1])
        assert _value(s, "amdgpu_dp_container_hbm_used_bytes", **lab) == 0  # given back at exit
        assert _value(s, "amdgpu_dp_container_hbm_peak_bytes", **lab) == 2000 * mib
        assert _value(s, "amdgpu_dp_container_hbm_processes", namespace="ml", pod="infer") == 0

        # The pod is gone: its file goes once it is two minutes old.
        pr.payload = _list_response([])
        time.sleep(2.1)
        _get(port, "/metrics")
        assert os.path.exists(host)  # too young
        os.utime(host, (time.time() - 300, time.time() - 300))
        s = _parse(_get(port, "/metrics")[1])
        assert not os.path.exists(host)
        assert not any(n == "amdgpu_dp_container_hbm_used_bytes" for (n, _) in s)
    finally:
        if holder:
            holder.kill()
        pr.stop()
        d.stop()
        k.stop()


def test_container_hbm_files_without_pod_resources_and_tampered(scratch):
    """Without PodResources a grant file is reported by its own device IDs
    (allocation label). The files are the containers' to write: a symlink, a
    non-regular file or a bad header is skipped, IDs that do not hash to the
    file name are not believed, and a file grown past its size is trimmed."""
    import subprocess
    shim, check = _preloadable_shim()
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=[
        "--metrics-addr", "127.0.0.1:0", "--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack",
        "--enforce-memory-units", "--memcap-lib", shim]).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        first = c.allocate(ids[:2]).container_responses[0]
        second = c.allocate(ids[2:3]).container_responses[0]
        c.close()
        path = lambda r: [m.host_path for m in r.mounts if m.container_path == "/run/amdgpu-dp/memcap"][0]
        p1, p2 = path(first), path(second)
        assert _wait_file(p1) and _wait_file(p2)
        key1 = os.path.basename(p1).split(".")[0]
        s = _parse(_get(port, "/metrics")[1])
        g0 = ids[0].split("-replica-")[0]
        assert _value(s, "amdgpu_dp_container_hbm_granted_bytes", allocation=key1, device=g0) == 2000 << 20
        assert _value(s, "amdgpu_dp_container_hbm_used_bytes", allocation=key1) == 0

        usage_dir = os.path.dirname(p1)
        # The second container rewrites its IDs to claim the first one's devices... 
        with open(p2, "r+b") as f:
            f.seek(24 + 4 * 64 * 8)  # ids[] after the header words and the four per-device columns
            f.write(b"somebody-else,")
        # ... a link and a directory posing as grant files ...
        os.symlink("/etc/passwd", os.path.join(usage_dir, "00000000000000aa.memcap"))
        os.mkdir(os.path.join(usage_dir, "00000000000000bb.memcap"))
        # ... and the first one grows its file.
        with open(p1, "r+b") as f:
            f.truncate(1 << 30)
        s = _parse(_get(port, "/metrics")[1])
        allocs = {dict(ls).get("allocation") for (n, ls), _ in s.items() if n == "amdgpu_dp_container_hbm_used_bytes"}
        assert allocs == {key1}
        assert os.path.getsize(p1) < 1 << 20  # trimmed back to the accounting area
        assert os.path.islink(os.path.join(usage_dir, "00000000000000aa.memcap"))  # not followed, not removed
        assert open("/etc/passwd").read()  # untouched
        # The trimmed file still works for the shim.
        env = dict(os.environ, LD_PRELOAD=" ".join(x for x in (os.environ.get("LD_PRELOAD", ""), shim) if x),
                   AMD_GPU_MEMORY_LIMIT_MIB="2000", ADP_MEMCAP_FILE=p1)
        r = subprocess.run([check, "try", "0", "1500"], capture_output=True,
                           text=True, timeout=30, env=env)
        assert r.returncode == 0 and '"rc": 0' in r.stdout.splitlines()[0], r.stdout
        s = _parse(_get(port, "/metrics")[1])
        assert _value(s, "amdgpu_dp_container_hbm_peak_bytes", allocation=key1) == 1500 << 20
    finally:
        d.stop()
        k.stop()


def test_status_cli_reads_metrics(served):
    """`python -m k8s_gpu_sharing_plugin_amd status URL`: the resource line with
    devices / healthy / allocatable / registered / RPC counts / residency, and
    exit 1 with an UNHEALTHY line once a device fails."""
    import subprocess
    import sys
    d, k, c, port, fifo = served
    q, call = c.watch()
    ids = [x.ID for x in q.get(timeout=5).devices]
    for _ in range(3):
        c.allocate([ids[0]])
    d.wait_log("health monitor watching")
    url = f"http://127.0.0.1:{port}/metrics"
    cmd = [sys.executable, "-m", "k8s_gpu_sharing_plugin_amd", "status", url]
    deadline = time.time() + 5
    while True:  # registered is marked just after Register() reaches the kubelet
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=60)
        if r.returncode == 0 or time.time() > deadline:
            break
        time.sleep(0.1)
    assert r.returncode == 0, r.stdout + r.stderr
    line = next(ln for ln in r.stdout.splitlines() if ln.startswith("amd.com/sharedgpu"))
    cols = line.split()
    assert cols[1:5] == ["2", "2", "6", "yes"] and int(cols[5]) == 3, line
    assert re.search(r"\d+\.\d / \d+\.\d$", line), line  # residency p50 / p99 at 100 ns (from /stats)
    health = next(ln for ln in r.stdout.splitlines() if ln.startswith("health: "))
    assert re.match(r"health: events (on|off \(polling\)), monitor loop \d+\.\d s ago", health), health
    fd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
    os.write(fd, b"1 3 pre-reset\n")
    os.close(fd)
    deadline = time.time() + 5
    while True:
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=60)
        if r.returncode == 1 or time.time() > deadline:
            break
        time.sleep(0.1)
    assert r.returncode == 1 and "UNHEALTHY amd.com/sharedgpu" in r.stdout, r.stdout
    call.cancel()


def test_stats_endpoint_is_json(served):
    """GET /stats: the SIGUSR1 counters as one JSON document (plugins with
    RPC counts and the residency histogram, health counters, restarts)."""
    import json
    d, k, c, port, _ = served
    q, call = c.watch()
    ids = [x.ID for x in q.get(timeout=5).devices]
    for _ in range(4):
        c.allocate([ids[0]])
    with urllib.request.urlopen(f"http://127.0.0.1:{port}/stats", timeout=5) as r:
        assert r.headers["Content-Type"] == "application/json"
        st = json.loads(r.read())
    (p,) = [p for p in st["plugins"] if p["resource"] == "amd.com/sharedgpu"]
    assert p["allocate_calls"] == 4 and p["devices"] == 2 and p["advertised"] == 6
    assert sum(n for _, n in p["residency_100ns"]) >= 4 and p["residency_p50_us"] > 0
    assert st["health"]["events"] in ("on", "off", "not started") and st["restarts"] >= 1
    call.cancel()
    # only GET: a scraper that POSTs is told so, and an unknown path is a 404
    req = urllib.request.Request(f"http://127.0.0.1:{port}/metrics", data=b"x", method="POST")
    try:
        urllib.request.urlopen(req, timeout=5)
        raise AssertionError("POST accepted")
    except urllib.error.HTTPError as e:
        assert e.code == 405 and e.read() == b"only GET\n"
    assert _get(port, "/nosuch")[0] == 404


def test_metrics_listens_on_every_address_given(scratch):
    """--metrics-addr takes a comma-separated list (the chart: the pod IP for
    Prometheus and loopback for kubectl port-forward and in-pod tools, which
    dial 127.0.0.1): every address answers; one that cannot be bound fails the
    start instead of serving half."""
    import socket
    import subprocess
    import urllib.request
    with socket.socket() as s0:
        s0.bind(("127.0.0.1", 0))
        port = s0.getsockname()[1]
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(1), args=[
        "--metrics-addr", f"127.0.0.2:{port}, 127.0.0.1:{port}"]).start()
    try:
        assert f"on port {port} (and /stats) at 127.0.0.2:{port}" in d.wait_log("serving /metrics")
        for host in ("127.0.0.1", "127.0.0.2"):
            with urllib.request.urlopen(f"http://{host}:{port}/metrics", timeout=5) as r:
                assert b"amdgpu_dp_build_info" in r.read()
    finally:
        d.stop()
        k.stop()
    r = subprocess.run([harness.DAEMON, "--device-plugin-path", scratch, "--metrics-addr",
                        f"127.0.0.1:{port},not-an-address:x"], capture_output=True, text=True, timeout=30,
                       env=harness.Daemon(scratch, fixtures.node(1)).env)
    assert r.returncode == 1 and "invalid --metrics-addr 'not-an-address:x'" in r.stdout + r.stderr

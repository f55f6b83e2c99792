"""Every deliberate deviation from the reference's kubelet-facing contract,
pinned to the value chosen here (docs/PARITY.md, "Deliberate deviations").

The reference is /root/reference/cmd/nvidia-device-plugin/server.go; each test
names the lines whose behaviour it departs from and asserts what this plugin
does instead. Behaviour that matches the reference exactly is pinned too where
a deviation sits next to it (the unknown-device error text, the envvar list
order), so a change to either side is seen.
"""

import os

import grpc
import pytest

from k8s_gpu_sharing_plugin_amd import REPO_ROOT
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet


class Served:
    def __init__(self, scratch, fx=None, args=()):
        self.k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        self.d = harness.Daemon(scratch, fx or fixtures.node(2), args=list(args)).start()
        self.reg = self.k.wait_registration()
        self.c = kubelet.PluginClient(os.path.join(scratch, self.reg.endpoint))
        q, call = self.c.watch()
        self.ids = [x.ID for x in q.get(timeout=5).devices]
        call.cancel()

    def close(self):
        self.c.close()
        self.d.stop()
        self.k.stop()


@pytest.fixture
def served(scratch):
    made = []

    def make(**kw):
        s = Served(scratch, **kw)
        made.append(s)
        return s
    yield make
    for s in made:
        s.close()


@pytest.mark.parametrize("args", [["--partition-strategy", "single"], ["--partition-strategy", "mixed"],
                                  ["--partition-strategy", "none"]])
def test_preferred_allocation_is_always_offered(served, args):
    """Reference server.go:231,245: GetPreferredAllocationAvailable only with an
    allocation policy or replicas -- false for MIG resources (single, mixed)
    without replicas, and GetPreferredAllocation then errors "not implemented in
    this case" (server.go:301-303). Here it is always true, in Register and in
    GetDevicePluginOptions alike, and GetPreferredAllocation answers for
    partitions and whole GPUs with IDs from the available set."""
    fx = fixtures.node(2, ["CPX", "CPX"], memory="NPS2") if "none" not in args else None
    s = served(fx=fx, args=args)
    assert s.reg.options.get_preferred_allocation_available is True
    opts = s.c.options()
    assert opts.get_preferred_allocation_available is True and opts.pre_start_required is False
    got = list(s.c.preferred(s.ids, (), 2).container_responses[0].deviceIDs)
    assert len(got) == 2 and set(got) <= set(s.ids)
    if "none" not in args:
        # partitions of one GPU together: the advertised list holds each GPU's 8
        # CPX partitions in a row (unit order)
        gpu_of = {i: n // 8 for n, i in enumerate(s.ids[:16])}
        for k in (2, 8):
            got = list(s.c.preferred(s.ids[:16], (), k).container_responses[0].deviceIDs)
            assert len({gpu_of[i] for i in got}) == 1, (k, got)


def test_prestart_is_required_only_when_asked(served):
    """Reference server.go:356-358: PreStartContainer is a no-op and never
    requested. Here too, unless --prestart-health-check (then requested, and it
    refuses Unhealthy devices)."""
    s = served(args=["--prestart-health-check"])
    assert s.reg.options.pre_start_required is True and s.c.options().pre_start_required is True


def test_device_specs_are_passed_by_default(served):
    """Reference main.go:73-78: --pass-device-specs defaults to false (NVIDIA's
    runtime hook creates the nodes from NVIDIA_VISIBLE_DEVICES). On AMD nothing
    reads an env var: the device nodes are what makes a GPU usable, so the
    default is true -- /dev/kfd plus the GPU's render node."""
    s = served()
    resp = s.c.allocate([s.ids[0]]).container_responses[0]
    paths = sorted(d.container_path for d in resp.devices)
    assert paths[0] == "/dev/dri/renderD128" and "/dev/kfd" in paths
    assert all(d.permissions == "rw" for d in resp.devices)


def test_device_list_envvar_and_volume_mount_root_are_amd_names(served, scratch):
    """Reference server.go:37-53: NVIDIA_VISIBLE_DEVICES and
    /var/run/nvidia-container-devices. Here AMD_VISIBLE_DEVICES and
    /var/run/amd-container-devices, same shapes; with the uuid strategy the
    list is sorted (stripReplicas sorts, replica.go:32-45), duplicates of one
    GPU's replicas collapse."""
    s = served(args=["--resource-config", "gpu:gpu:2"])
    ids = sorted(s.ids, reverse=True)
    env = dict(s.c.allocate(ids).container_responses[0].envs)
    uuids = sorted({i.split("-replica-")[0] for i in ids})
    assert env["AMD_VISIBLE_DEVICES"] == ",".join(uuids)
    s.close()
    os.makedirs(scratch + "v")
    s2 = Served(scratch + "v", args=["--device-list-strategy", "volume-mounts"])
    try:
        resp = s2.c.allocate([s2.ids[0]]).container_responses[0]
        assert dict(resp.envs)["AMD_VISIBLE_DEVICES"] == "/var/run/amd-container-devices"
        assert [(m.container_path, m.host_path) for m in resp.mounts] == [
            ("/var/run/amd-container-devices/" + s2.ids[0], "/dev/null")]
    finally:
        s2.close()


def test_unknown_device_error_matches_the_reference(served):
    """Same text as server.go:320-323 (kept: tooling greps kubelet events for it)."""
    s = served()
    with pytest.raises(grpc.RpcError) as e:
        s.c.allocate(["no-such-gpu"])
    assert e.value.details() == "invalid allocation request for 'amd.com/gpu': unknown device: no-such-gpu"


def test_events_unavailable_do_not_mark_devices_unhealthy(scratch):
    """Reference nvidia.go:218-223: a device whose event registration fails is
    marked Unhealthy (on NVIDIA that meant a pre-Kepler GPU). Here it stays
    Healthy and health falls back to polling (an unprivileged pod cannot open
    /dev/kfd; that says nothing about the GPU)."""
    fx = dict(fixtures.node(2), events_supported=False)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, env={"DP_HEALTH_POLL_MS": "100"}).start()
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        q, call = c.watch()
        assert [x.health for x in q.get(timeout=5).devices] == ["Healthy", "Healthy"]
        d.wait_log("health poll #1")
        assert q.empty()
        call.cancel()
        c.close()
    finally:
        d.stop()
        k.stop()


def test_unhealthy_allocation_is_counted_not_silent(scratch):
    """Reference server.go:316-353 allocates an Unhealthy device without a word.
    Here the same (the kubelet's view may be a moment old) with a warning and
    amdgpu_dp_unhealthy_allocations_total; --reject-unhealthy refuses it."""
    fifo = os.path.join(scratch + ".fixture", "events")
    os.makedirs(os.path.dirname(fifo), exist_ok=True)
    os.mkfifo(fifo)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), event_fifo=fifo, env={"DP_HEALTH_POLL_MS": "100"}).start()
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        q, call = c.watch()
        ids = [x.ID for x in q.get(timeout=5).devices]
        d.wait_log("health monitor watching")
        fd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
        os.write(fd, b"0 3 reset\n")
        os.close(fd)
        assert [x.health for x in q.get(timeout=5).devices] == ["Unhealthy", "Healthy"]
        c.allocate([ids[0]])  # allocated anyway, as the reference does
        assert "is Unhealthy (allocated anyway" in d.wait_log("allocated anyway")
        call.cancel()
        c.close()
    finally:
        d.stop()
        k.stop()


def _chart_pod(values=None):
    import sys
    import yaml
    sys.path.insert(0, os.path.join(REPO_ROOT, "tools"))
    import helm_render
    out = helm_render.render(values or {})
    ds = [d for d in yaml.safe_load_all(out["daemonset.yaml"]) if d and d.get("kind") == "DaemonSet"][0]
    spec = ds["spec"]["template"]["spec"]
    containers = spec.get("initContainers", []) + spec["containers"]
    host_paths = {v["name"]: v["hostPath"]["path"] for v in spec["volumes"] if v.get("hostPath")}
    return containers, host_paths, helm_render.render_notes(values or {})


def test_default_install_security_posture_is_the_documented_deviation():
    """docs/PARITY.md rows "Privileged container by default" and "Writable host
    directory by default": the reference's default install is one drop-ALL
    container with one hostPath, the kubelet's device-plugin directory
    (/root/reference/deployments/helm/nvidia-device-plugin/templates/daemonset.yml:80-104).
    Here the default is exactly one privileged container -- the event relay --
    and the plugin container drops everything; the host paths are the ones
    listed, /var/lib/amdgpu-device-plugin the only one beyond the kubelet's that
    is written. The install notes say so, with the opt-outs; with both opt-outs
    nothing is privileged and nothing of the host is written but the kubelet's
    directory."""
    containers, host_paths, notes = _chart_pod()
    privileged = [c["name"] for c in containers if (c.get("securityContext") or {}).get("privileged")]
    assert privileged == ["event-relay"], privileged
    plugin = [c for c in containers if c["name"] != "event-relay"]
    assert len(plugin) == 1 and plugin[0]["securityContext"]["capabilities"] == {"drop": ["ALL"]}
    assert plugin[0]["securityContext"]["allowPrivilegeEscalation"] is False
    assert host_paths == {"device-plugin": "/var/lib/kubelet/device-plugins", "sys": "/sys", "dev": "/dev",
                          "health-state": "/var/lib/amdgpu-device-plugin"}, host_paths
    writable = {m["name"] for c in containers for m in c.get("volumeMounts", [])
                if m["name"] in host_paths and not m.get("readOnly")}
    assert writable == {"device-plugin", "dev", "health-state"}, writable
    assert '"event-relay" container runs privileged' in notes and "healthEvents=false" in notes
    assert "/var/lib/amdgpu-device-plugin is mounted writable" in notes and "healthState.enabled=false" in notes
    parity = open(os.path.join(REPO_ROOT, "docs", "PARITY.md")).read()
    assert "| Privileged container by default |" in parity and "| Writable host directory by default |" in parity

    containers, host_paths, notes = _chart_pod({"healthEvents": False, "healthState": {"enabled": False}})
    assert not [c for c in containers if (c.get("securityContext") or {}).get("privileged")]
    assert [c["name"] for c in containers] == ["amdgpu-device-plugin"]
    assert host_paths == {"device-plugin": "/var/lib/kubelet/device-plugins", "sys": "/sys", "dev": "/dev"}
    assert "privileged" not in notes

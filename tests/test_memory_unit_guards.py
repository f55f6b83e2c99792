"""What a memory unit is, said and guarded.

A memory-unit resource (resourceConfig replicas -1) advertises one ID per
unit of HBM. With --replica-cu-mask the unit becomes a CU slot -- one CU on
every XCD and its share of the HBM, ~9 GiB on an MI355X -- so the default
name "gpu-mem-gb" would promise 1 GB per unit and deliver nine. The daemon
warns about a gigabyte name over a non-gigabyte unit, publishes every
memory-unit resource's unit as node labels and /metrics, and -- because a
changed unit or replica count re-means IDs the kubelet's checkpoint still
holds for running pods -- logs an error and counts it when a restart changes
what a resource's IDs mean while PodResources shows them held.

Parity: the reference's unit is fixed (one replica per 1000 MiB,
/root/reference/cmd/nvidia-device-plugin/server.go:99-111) and it has none of
these checks; the chart default it is compared with is
/root/reference/deployments/helm/nvidia-device-plugin/values.yaml:13.
"""

import os
import re
import subprocess
import sys
import time

import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

from test_metrics import PodResourcesStub, _get, _list_response, _parse, _value


def _start(scratch, args, labels=None, pr_sock=None):
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    extra = ["--metrics-addr", "127.0.0.1:0"]
    if labels:
        extra += ["--node-labels-file", labels]
    if pr_sock:
        extra += ["--pod-resources-socket", pr_sock]
    d = harness.Daemon(scratch, fixtures.node(2), args=[*args, *extra]).start()
    port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
    return k, d, port


def _labels(path):
    deadline = time.time() + 5
    while not os.path.exists(path):
        assert time.time() < deadline
        time.sleep(0.02)
    return dict(line.split("=", 1) for line in open(path).read().splitlines() if line)


def test_cu_slot_units_under_a_gigabyte_name_warn_and_say_their_size(scratch):
    labels = scratch + ".labels"
    k, d, port = _start(scratch, ["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-cu-mask"], labels)
    try:
        log = d.wait_log("is named for gigabytes")
        line = [ln for ln in log.splitlines() if "is named for gigabytes" in ln][0]
        m = re.search(r"one unit is (\d+) MiB \(cu-slot units", line)
        assert m and int(m.group(1)) > 4000, line
        unit = int(m.group(1))
        assert "gpu:gpu-slot:-1" in line and "amd.com/gpu-mem-gb.memory-unit-mib" in line
        assert f"'amd.com/gpu-mem-gb' units of {unit} MiB (cu-slot)" in log
        lab = _labels(labels)
        assert lab["amd.com/gpu-mem-gb.memory-unit"] == "cu-slot"
        assert lab["amd.com/gpu-mem-gb.memory-unit-mib"] == str(unit)
        s = _parse(_get(port, "/metrics")[1])
        units = [v for (n, ls), v in s.items() if n == "amdgpu_dp_memory_unit_mib"]
        assert units == [unit, unit]
        assert all(dict(ls)["kind"] == "cu-slot" for (n, ls) in s if n == "amdgpu_dp_memory_unit_mib")
    finally:
        d.stop()
        k.stop()


def test_mib_units_and_honest_names_do_not_warn(scratch):
    labels = scratch + ".labels"
    for args, name, kind, mib in [(["--resource-config", "gpu:gpu-mem-gb:-1"], "gpu-mem-gb", "mib", "1000"),
                                  (["--resource-config", "gpu:gpu-slot:-1", "--replica-cu-mask"], "gpu-slot",
                                   "cu-slot", None)]:
        k, d, port = _start(scratch, args, labels)
        try:
            d.wait_log("replicating device")
            lab = _labels(labels)
            assert lab[f"amd.com/{name}.memory-unit"] == kind
            if mib:
                assert lab[f"amd.com/{name}.memory-unit-mib"] == mib
            assert "is named for gigabytes" not in d.log()
        finally:
            d.stop()
            k.stop()


def _config(path, unit):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write("version: v1\nflags:\n  resourceConfig: gpu:gpu-mem-gb:-1\n  replicaCuMask: true\n"
                f"  autoReplicaUnit: {unit}\n")
    os.rename(tmp, path)


def test_changing_the_unit_under_live_grants_is_an_error(scratch):
    """A running pod holds memory-unit IDs; the config changes the unit from
    MiB to CU slots: the new generation advertises 32 IDs per GPU where there
    were ~290, so some held IDs no longer exist and the rest mean 9 GiB where
    the pod got 1000 MiB. Logged as an error, counted, and the held IDs that
    no longer exist show in amdgpu_dp_stale_allocated_ids. A change with no
    pod holding IDs is only noted. The layout outlives the process too: a
    daemon restarted with another unit checks against the last one."""
    pr_sock = os.path.join(scratch + ".fixture", "pod-resources.sock")
    os.makedirs(os.path.dirname(pr_sock), exist_ok=True)
    pr = PodResourcesStub(pr_sock)
    cfg = os.path.join(scratch + ".fixture", "config.yaml")
    _config(cfg, "mib")
    k, d, port = _start(scratch, ["--config-file", cfg], pr_sock=pr_sock)
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        c.close()
        assert len(ids) > 200
        res = "amd.com/gpu-mem-gb"
        held = [ids[0], ids[1], ids[100], ids[101]]  # replicas 0, 1, 100, 101 of GPU 0
        pr.payload = _list_response([("ml", "train", "main", res, held)])
        _config(cfg, "auto")  # -> CU slots under replicaCuMask
        log = d.wait_log("what its IDs mean changed while")
        line = [ln for ln in log.splitlines() if "what its IDs mean changed while" in ln][0]
        assert " E daemon:" in line and "4 of them are held by 1 running pod(s)" in line and "Drain the node" in line
        s = _parse(_get(port, "/metrics")[1])
        assert _value(s, "amdgpu_dp_replica_layout_changes_with_live_allocations_total", resource=res) == 1
        assert _value(s, "amdgpu_dp_stale_allocated_ids", resource=res) == 2  # replicas 100, 101 are gone
        # the status CLI says so, with what one unit now is, and fails
        st = subprocess.run([sys.executable, "-m", "k8s_gpu_sharing_plugin_amd", "status",
                             f"http://127.0.0.1:{port}/metrics"], capture_output=True, text=True, timeout=60)
        assert st.returncode == 1, st.stdout + st.stderr
        assert f"STALE {res}: 2 ID(s) running pods hold are no longer advertised" in st.stdout, st.stdout
        assert re.search(rf"^{res}: one unit = \d+ MiB \(cu-slot\)$", st.stdout, re.M), st.stdout
        # no pod holds IDs any more: a change back is only noted
        pr.payload = _list_response([])
        _config(cfg, "mib")
        log = d.wait_log("no running container holds any")
        assert log.count("what its IDs mean changed while") == 1
        assert d.stop() == 0
        # the next process remembers the layout (<plugin dir>/amdgpu-dp/replica-layout)
        pr.payload = _list_response([("ml", "train", "main", res, held)])
        _config(cfg, "cu-slot")
        d = harness.Daemon(scratch, fixtures.node(2), args=["--config-file", cfg, "--metrics-addr", "127.0.0.1:0",
                                                            "--pod-resources-socket", pr_sock]).start()
        d.wait_log("what its IDs mean changed while")
    finally:
        d.stop()
        k.stop()
        pr.stop()


def test_a_resource_absent_for_a_while_keeps_its_layout(scratch):
    """A memory-unit resource leaves the config (the node serves another
    resource meanwhile) and comes back with another unit while a pod still
    holds its old IDs: still a change under live grants -- the last layout
    seen is kept while the resource is absent."""
    pr_sock = os.path.join(scratch + ".fixture", "pod-resources.sock")
    os.makedirs(os.path.dirname(pr_sock), exist_ok=True)
    pr = PodResourcesStub(pr_sock)
    cfg = os.path.join(scratch + ".fixture", "config.yaml")

    def write(rc, unit):
        tmp = cfg + ".tmp"
        with open(tmp, "w") as f:
            f.write(f"version: v1\nflags:\n  resourceConfig: {rc}\n  replicaCuMask: true\n"
                    f"  autoReplicaUnit: {unit}\n")
        os.rename(tmp, cfg)
    write("gpu:gpu-mem-gb:-1", "mib")
    k, d, port = _start(scratch, ["--config-file", cfg], pr_sock=pr_sock)
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        c.close()
        res = "amd.com/gpu-mem-gb"
        pr.payload = _list_response([("ml", "train", "main", res, [ids[0], ids[200]])])
        write("gpu:sharedgpu:4", "mib")  # the memory-unit resource is gone for now
        d.wait_log("'amd.com/sharedgpu': preferred allocation")
        layout = open(os.path.join(scratch, "amdgpu-dp", "replica-layout")).read()
        assert layout.count("amd.com/gpu-mem-gb\tmemory-units mib") == 1, layout  # remembered
        write("gpu:gpu-mem-gb:-1", "cu-slot")  # back, with another unit, the pod still running
        log = d.wait_log("what its IDs mean changed while")
        assert "'amd.com/gpu-mem-gb'" in [ln for ln in log.splitlines() if "what its IDs mean changed while" in ln][0]
        s = _parse(_get(port, "/metrics")[1])
        assert _value(s, "amdgpu_dp_replica_layout_changes_with_live_allocations_total", resource=res) == 1
    finally:
        d.stop()
        k.stop()
        pr.stop()


def test_a_layout_change_under_live_grants_can_wait_for_the_pods(scratch):
    """--defer-layout-changes: a config change that would re-mean IDs running
    pods hold does not apply while they run -- the current layout keeps being
    served (amdgpu_dp_deferred_layout_change says so) -- and applies by itself
    once they are gone, with no over-commit in between."""
    pr_sock = os.path.join(scratch + ".fixture", "pod-resources.sock")
    os.makedirs(os.path.dirname(pr_sock), exist_ok=True)
    pr = PodResourcesStub(pr_sock)
    cfg = os.path.join(scratch + ".fixture", "config.yaml")
    _config(cfg, "mib")
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=[
        "--config-file", cfg, "--metrics-addr", "127.0.0.1:0", "--pod-resources-socket", pr_sock,
        "--defer-layout-changes"], env={"ADP_DEFER_RECHECK_MS": "300"}).start()
    port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        c.close()
        res = "amd.com/gpu-mem-gb"
        pr.payload = _list_response([("ml", "train", "main", res, [ids[0], ids[100]])])
        _config(cfg, "auto")  # -> CU slots: what the held IDs mean would change
        log = d.wait_log("config change deferred")
        assert f"running pods hold IDs of '{res}'" in log
        time.sleep(1.0)  # three rechecks: still deferred, still the old layout
        assert "what its IDs mean changed while" not in d.log() and d.log().count("config change deferred") == 1
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        assert len(c.watch()[0].get(timeout=5).devices) == len(ids)
        c.close()
        s = _parse(_get(port, "/metrics")[1])
        assert _value(s, "amdgpu_dp_deferred_layout_change", resource=res) == 1
        st = subprocess.run([sys.executable, "-m", "k8s_gpu_sharing_plugin_amd", "status",
                             f"http://127.0.0.1:{port}/metrics"], capture_output=True, text=True, timeout=60)
        assert f"DEFERRED {res}: a config change waits" in st.stdout, st.stdout
        pr.payload = _list_response([])  # the pod ended
        reg = k.wait_registration(15)  # the change applied: the plugin restarts with it
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        assert len(c.watch()[0].get(timeout=5).devices) == 64  # 32 CU slots per GPU
        c.close()
        assert "deferred config change: reloaded config" in d.log()
        assert "what its IDs mean changed while" not in d.log()
        s = _parse(_get(port, "/metrics")[1])
        assert not [v for (n, ls), v in s.items() if n == "amdgpu_dp_deferred_layout_change"]
    finally:
        d.stop()
        k.stop()
        pr.stop()


def test_a_whole_gpu_resource_turned_into_replicas_waits_for_its_pods(scratch):
    """--defer-layout-changes, from a whole-GPU resource (no replicas, an empty
    layout) to time-slice replicas while a pod holds one GPU exclusively: the
    same GPU would be shared by new pods -- a re-meaning, deferred like any
    other (round-5 advice: an empty layout becoming non-empty is a change)."""
    pr_sock = os.path.join(scratch + ".fixture", "pod-resources.sock")
    os.makedirs(os.path.dirname(pr_sock), exist_ok=True)
    pr = PodResourcesStub(pr_sock)
    cfg = os.path.join(scratch + ".fixture", "config.yaml")

    def write(rc):
        tmp = cfg + ".tmp"
        with open(tmp, "w") as f:
            f.write(f"version: v1\nflags:\n  resourceConfig: {rc}\n")
        os.rename(tmp, cfg)
    write("gpu:gpu:1")
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=[
        "--config-file", cfg, "--metrics-addr", "127.0.0.1:0", "--pod-resources-socket", pr_sock,
        "--defer-layout-changes"], env={"ADP_DEFER_RECHECK_MS": "300"}).start()
    port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        c.close()
        assert len(ids) == 2 and not any("-replica-" in i for i in ids)
        res = "amd.com/gpu"
        pr.payload = _list_response([("ml", "train", "main", res, [ids[0]])])
        write("gpu:gpu:4")  # the held GPU would become 4 replicas, 3 of them for new pods
        log = d.wait_log("config change deferred")
        assert f"running pods hold IDs of '{res}'" in log
        time.sleep(0.8)
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        assert [x.ID for x in c.watch()[0].get(timeout=5).devices] == ids  # still whole GPUs
        c.close()
        assert _value(_parse(_get(port, "/metrics")[1]), "amdgpu_dp_deferred_layout_change", resource=res) == 1
        pr.payload = _list_response([])  # the pod ended
        reg = k.wait_registration(15)
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        assert len(c.watch()[0].get(timeout=5).devices) == 8
        c.close()
        assert "what its IDs mean changed while" not in d.log()
    finally:
        d.stop()
        k.stop()
        pr.stop()


@pytest.mark.parametrize("socket", ["none", "unreachable"])
def test_a_deferral_that_cannot_know_applies_and_says_so(scratch, socket):
    """--defer-layout-changes can only wait for pods the kubelet's PodResources
    API names: without its socket, or with one that does not answer, a change
    that re-means IDs applies (a config change is never blocked on an unknown)
    with a warning saying why."""
    cfg = os.path.join(scratch + ".fixture", "config.yaml")
    os.makedirs(os.path.dirname(cfg), exist_ok=True)

    def write(rc):
        with open(cfg + ".tmp", "w") as f:
            f.write(f"version: v1\nflags:\n  resourceConfig: {rc}\n")
        os.rename(cfg + ".tmp", cfg)
    write("gpu:gpu:2")
    args = ["--config-file", cfg, "--defer-layout-changes"]
    if socket == "none":
        args += ["--pod-resources-socket="]  # (its default is the kubelet's path)
    else:
        args += ["--pod-resources-socket", os.path.join(scratch + ".fixture", "nobody-listens.sock")]
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=args).start()
    try:
        reg = k.wait_registration()
        write("gpu:gpu:3")
        reg = k.wait_registration(15)  # applied
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        assert len(c.watch()[0].get(timeout=5).devices) == 6
        c.close()
        want = ("--defer-layout-changes needs the kubelet's PodResources socket; applying" if socket == "none"
                else "whether running pods hold IDs of the resources this change re-means is unknown")
        assert want in d.wait_log(want)
        assert "config change deferred" not in d.log()
    finally:
        d.stop()
        k.stop()

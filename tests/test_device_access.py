"""Device access of the plugin's own pod: what a device cgroup takes away.

The reference image gets its device nodes from the NVIDIA runtime
(NVIDIA_VISIBLE_DEVICES=all, /root/reference/deployments/container/
Dockerfile.ubuntu:32-33) and its chart escalates for MIG monitoring
(/root/reference/deployments/helm/nvidia-device-plugin/templates/
daemonset.yml:72-93). Here amdsmi's event notification opens /dev/kfd, which
the device cgroup of an unprivileged pod denies with EPERM even when /dev is a
hostPath mount. libadp_devcgroup_sim.so reproduces exactly that errno for
/dev/kfd and /dev/dri/*; on the MI355X box, with the real libamd_smi, the same
denial leaves enumeration, ECC, retired pages, process list and partition
queries working and fails event registration, vram_info and asic_info
(profiles/r3/access/access_summary.txt; tests/test_gpu.py::
test_health_under_device_cgroup_denial). The daemon says so and why.
"""

import json
import os
import re
import subprocess

from k8s_gpu_sharing_plugin_amd import BUILD_DIR, DAEMON, MOCK_LIB
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

from test_metrics import _get, _parse, _value

SIM = os.path.join(BUILD_DIR, "libadp_devcgroup_sim.so")


def _preload(*libs):
    return " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), *libs) if x)


def test_events_off_names_the_device_cgroup(scratch):
    fx = dict(fixtures.node(2), events_open_kfd=True)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fx, args=["--metrics-addr", "127.0.0.1:0"],
                       env={"LD_PRELOAD": _preload(SIM), "DP_HEALTH_POLL_MS": "100"}).start()
    try:
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics")).group(1))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        law = c.watch()[0].get(timeout=5)
        assert {x.health for x in law.devices} == {"Healthy"} and len(law.devices) == 2  # still served
        log = d.wait_log("health poll #1")
        assert "device access: Operation not permitted: /dev/kfd, /dev/dri/renderD128" in log
        assert "device cgroup" in log
        events = [ln for ln in log.splitlines() if "events off:" in ln][0]
        assert "/dev/kfd not openable (EPERM)" in events and "privileged" in events
        s = _parse(_get(port, "/metrics")[1])
        assert _value(s, "amdgpu_dp_device_node_openable", node="/dev/kfd") == 0
        assert _value(s, "amdgpu_dp_health_events_enabled") == 0
        assert _value(s, "amdgpu_dp_health_polls_total") >= 1  # polling carries on
        c.close()
    finally:
        d.stop()
        k.stop()


def test_health_events_can_be_turned_off(scratch):
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(1), args=["--health-events=false"],
                       env={"DP_HEALTH_POLL_MS": "100"}).start()
    try:
        k.wait_registration()
        log = d.wait_log("health monitor watching")
        assert "event notification off by configuration (--health-events=false)" in log
        assert "events off:" not in log  # no denial to explain: nothing was tried
        assert "(events off, poll every 100 ms)" in log
    finally:
        d.stop()
        k.stop()


def test_smi_report_shows_what_the_denial_breaks(tmp_path):
    fx = fixtures.write(dict(fixtures.node(1), events_open_kfd=True), str(tmp_path))
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=fx)
    run = lambda e: json.loads(subprocess.run([DAEMON, "--device-plugin-path", str(tmp_path), "--smi-report"],
                                              capture_output=True, text=True, timeout=30, env=e, check=True).stdout)
    free = run(env)
    denied = run(dict(env, LD_PRELOAD=_preload(SIM)))
    (p_free,), (p_denied,) = free["processors"], denied["processors"]
    assert p_free["event_notification_init"]["status"] == 0
    assert p_denied["event_notification_init"]["status"] == 10  # AMDSMI_STATUS_NO_PERM
    assert p_denied["uuid"]["status"] == 0 and p_denied["total_ecc_count"]["status"] == 0
    assert denied["enumeration"] == "ok"
    assert {a["node"]: a["errno"] for a in denied["device_access"]} == {"/dev/kfd": 1, "/dev/dri/renderD128": 1}
    assert all(a["error"] == "Operation not permitted" for a in denied["device_access"])

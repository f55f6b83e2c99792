"""The helm chart, rendered: valid Kubernetes objects for every values combination.

No helm binary exists in the image, so tools/helm_render.py implements the Go
template + sprig subset the chart uses; these tests render the chart with the
default values and with each feature switch, parse the output as YAML and
check the DaemonSet: env names the daemon understands, every volumeMount backed
by a volume, health state / metrics / NFD / reference value names wired up.

Parity: the reference chart (deployments/helm/nvidia-device-plugin/templates/
daemonset.yml:15-106) renders the same DaemonSet shape from the same keys.
"""

import os
import subprocess
import sys

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import helm_render  # noqa: E402

from k8s_gpu_sharing_plugin_amd import DAEMON  # noqa: E402


def daemon_envs():
    text = subprocess.run([DAEMON, "--help"], capture_output=True, text=True, check=True).stdout
    names = set()
    for tok in text.replace("(", " ").replace(",", " ").replace(")", " ").split():
        if tok.isupper() and "_" in tok:
            names.add(tok)
    # environment-only settings documented in docs/USER_GUIDE.md
    # POD_IP: the downward API value the kubelet expands into DP_METRICS_ADDR
    return names | {"DP_DISABLE_HEALTHCHECKS", "DP_HEALTH_POLL_MS", "DP_MAX_RETIRED_PAGES", "ADP_LOG_LEVEL",
                    "ADP_LOG_FORMAT", "POD_IP"}


def daemonset(values=None):
    out = helm_render.render(values)
    docs = [d for d in yaml.safe_load_all(out["daemonset.yaml"]) if d]
    assert len(docs) == 1
    return docs[0]


def container(ds, name="amdgpu-device-plugin"):
    (c,) = [c for c in ds["spec"]["template"]["spec"]["containers"] if c["name"] == name]
    return c


def relay(ds):
    cs = [c for c in ds["spec"]["template"]["spec"]["containers"] if c["name"] == "event-relay"]
    return cs[0] if cs else None


def env(ds):
    return {e["name"]: e.get("value") for e in container(ds)["env"]}


def check_consistent(ds):
    spec = ds["spec"]["template"]["spec"]
    vols = {v["name"] for v in spec["volumes"]}
    for c in spec["containers"]:
        mounts = {m["name"] for m in c["volumeMounts"]}
        assert mounts <= vols, (c["name"], mounts - vols)
    assert set(env(ds)) <= daemon_envs(), set(env(ds)) - daemon_envs()
    assert spec["priorityClassName"] == "system-node-critical"
    labels = ds["spec"]["template"]["metadata"]["labels"]
    if ds["apiVersion"] == "apps/v1":
        assert ds["spec"]["selector"]["matchLabels"].items() <= labels.items()


def test_defaults_render_a_valid_daemonset():
    ds = daemonset()
    check_consistent(ds)
    assert ds["apiVersion"] == "apps/v1" and ds["kind"] == "DaemonSet"
    assert ds["metadata"]["name"] == "amdgpu-amd-gpu-device-plugin"
    e = env(ds)
    assert e["PARTITION_STRATEGY"] == "none" and e["RESOURCE_CONFIG"] == "gpu:gpu-mem-gb:-1"
    assert e["REPLICA_POLICY"] == "auto" and e["FAIL_ON_INIT_ERROR"] == "true"
    assert e["AUTO_REPLICA_UNIT"] == "auto"
    # health state on by default: env + hostPath volume
    assert e["DP_HEALTH_STATE_FILE"] == "/var/lib/amdgpu-device-plugin/health.state"
    assert e["DP_DRAIN_FILE"] == "/var/lib/amdgpu-device-plugin/drain"
    vol = {v["name"]: v for v in ds["spec"]["template"]["spec"]["volumes"]}["health-state"]
    assert vol["hostPath"] == {"path": "/var/lib/amdgpu-device-plugin", "type": "DirectoryOrCreate"}
    assert container(ds)["image"] == "amdgpu-device-plugin:0.1.0"
    # health events on by default through the privileged event relay: the
    # plugin container itself is drop-ALL (privilege separation)
    assert e["DP_HEALTH_EVENTS"] == "true"
    assert e["DP_HEALTH_EVENT_SOCKET"] == "/run/amdgpu-dp-events/events.sock"
    sc = container(ds)["securityContext"]
    assert sc == {"allowPrivilegeEscalation": False, "readOnlyRootFilesystem": True,
                  "capabilities": {"drop": ["ALL"]}}, sc
    r = relay(ds)
    # both write only to mounted volumes (tests/test_chart_layout.py, on real amdsmi too)
    assert r["securityContext"] == {"privileged": True, "readOnlyRootFilesystem": True}
    assert r["args"] == ["--event-relay", "--health-event-socket", "/run/amdgpu-dp-events/events.sock"]
    assert not r.get("ports")  # no network-facing input
    # its liveness: the relay greets on its socket and its event wait is not stuck
    assert r["livenessProbe"]["exec"]["command"] == ["/usr/bin/amdgpu-device-plugin", "--relay-ping",
                                                     "--health-event-socket",
                                                     "/run/amdgpu-dp-events/events.sock"]
    shared = {m["name"]: m["mountPath"] for m in r["volumeMounts"]}
    assert shared["event-socket"] == "/run/amdgpu-dp-events"
    assert {m["name"]: m["mountPath"] for m in container(ds)["volumeMounts"]}["event-socket"] == "/run/amdgpu-dp-events"
    vols = {v["name"]: v for v in ds["spec"]["template"]["spec"]["volumes"]}
    assert vols["event-socket"]["emptyDir"]["medium"] == "Memory"
    assert e["DP_MAX_RETIRED_PAGES"] == "-1" and e["DP_LOOP_AFFINITY"] == "none"
    assert "livenessProbe" not in container(ds)


def test_health_events_off_runs_unprivileged():
    """healthEvents: false -> drop ALL, and the daemon is told events are off
    (it polls; it does not try /dev/kfd and log a denial)."""
    ds = daemonset({"healthEvents": False})
    check_consistent(ds)
    sc = container(ds)["securityContext"]
    assert sc["allowPrivilegeEscalation"] is False and sc["capabilities"]["drop"] == ["ALL"]
    assert env(ds)["DP_HEALTH_EVENTS"] == "false" and "DP_HEALTH_EVENT_SOCKET" not in env(ds)
    assert relay(ds) is None  # no privileged container at all
    assert "event-socket" not in {v["name"] for v in ds["spec"]["template"]["spec"]["volumes"]}
    # an explicit securityContext always wins; compat mode is privileged whatever healthEvents says
    custom = {"runAsUser": 0, "capabilities": {"add": ["SYS_ADMIN"]}}
    assert container(daemonset({"securityContext": custom}))["securityContext"] == custom
    compat = daemonset({"compatWithCPUManager": True})
    assert container(compat)["securityContext"] == {"privileged": True, "readOnlyRootFilesystem": True}
    assert relay(compat) is None and "DP_HEALTH_EVENT_SOCKET" not in env(compat)  # events in-process


@pytest.mark.parametrize("value,rendered", [(0, "0"), (-1, "-1"), (25, "25"), (None, "-1")])
def test_max_retired_pages_renders_zero_as_off(value, rendered):
    """0 means off: sprig's `default` would have turned it into -1 (the driver's threshold)."""
    assert env(daemonset({"maxRetiredPages": value}))["DP_MAX_RETIRED_PAGES"] == rendered


def test_driver_hbm_check_mounts_the_hosts_proc():
    """enforceMemoryUnits + metrics: the driver-side grant check reads the
    host's processes through a read-only hostPath /proc at /host/proc -- in the
    event relay (the pod's privileged container), so the daemon keeps no
    capability at all; without the relay the daemon reads them itself and gets
    CAP_SYS_PTRACE for it."""
    ds = daemonset({"enforceMemoryUnits": True, "metrics": {"enabled": True}})
    check_consistent(ds)
    e = env(ds)
    assert e["DP_DRIVER_HBM_POLL_MS"] == "10000" and e["DP_DRIVER_HBM_SLACK_MIB"] == "512"
    assert "DP_HOST_PROC" not in e and e["DP_HEALTH_EVENT_SOCKET"]
    assert container(ds)["securityContext"] == {"allowPrivilegeEscalation": False, "readOnlyRootFilesystem": True,
                                                "capabilities": {"drop": ["ALL"]}}
    assert "host-proc" not in {m["name"] for m in container(ds)["volumeMounts"]}
    r = relay(ds)
    assert {x["name"]: x["value"] for x in r["env"]}["DP_HOST_PROC"] == "/host/proc"
    mounts = {m["name"]: m for m in r["volumeMounts"]}
    assert mounts["host-proc"] == {"name": "host-proc", "mountPath": "/host/proc", "readOnly": True}
    # the grants' accounting files, at the path the daemon names them by
    assert mounts["device-plugin"] == {"name": "device-plugin", "mountPath": "/var/lib/kubelet/device-plugins",
                                       "readOnly": True}
    vols = {v["name"]: v for v in ds["spec"]["template"]["spec"]["volumes"]}
    assert vols["host-proc"]["hostPath"]["path"] == "/proc"
    # without the relay (health events off) the daemon scans: CAP_SYS_PTRACE and nothing else
    solo = daemonset({"enforceMemoryUnits": True, "metrics": {"enabled": True}, "healthEvents": False})
    check_consistent(solo)
    assert relay(solo) is None and env(solo)["DP_HOST_PROC"] == "/host/proc"
    (m,) = [m for m in container(solo)["volumeMounts"] if m["name"] == "host-proc"]
    assert m == {"name": "host-proc", "mountPath": "/host/proc", "readOnly": True}
    assert container(solo)["securityContext"]["capabilities"] == {"drop": ["ALL"], "add": ["SYS_PTRACE"]}
    for vals in ({"enforceMemoryUnits": True}, {"metrics": {"enabled": True}},
                 {"enforceMemoryUnits": True, "metrics": {"enabled": True}, "driverHbmCheck": {"enabled": False}}):
        off = daemonset(vals)
        assert env(off)["DP_DRIVER_HBM_POLL_MS"] == "0" and "DP_HOST_PROC" not in env(off)
        assert "host-proc" not in {v["name"] for v in off["spec"]["template"]["spec"]["volumes"]}
        assert container(off)["securityContext"]["capabilities"] == {"drop": ["ALL"]}
        assert "DP_HOST_PROC" not in {x["name"] for x in relay(off)["env"]}


def test_loop_affinity_value():
    assert env(daemonset({"loopAffinity": "peer-l3"}))["DP_LOOP_AFFINITY"] == "peer-l3"


def test_health_state_can_be_turned_off():
    ds = daemonset({"healthState": {"enabled": False}, "rejectUnhealthy": True})
    check_consistent(ds)
    assert "DP_HEALTH_STATE_FILE" not in env(ds)
    assert env(ds)["DP_REJECT_UNHEALTHY"] == "true"
    assert "health-state" not in {v["name"] for v in ds["spec"]["template"]["spec"]["volumes"]}


def test_sharing_and_health_gate_switches():
    """enforceMemoryUnits / replicaHbmShare / prestartHealthCheck reach the
    daemon; the shim is installed under the device-plugin dir, which must be
    mounted at its host path (the runtime bind-mounts that host path into pods)."""
    ds = daemonset({"enforceMemoryUnits": True, "replicaHbmShare": True, "prestartHealthCheck": True})
    check_consistent(ds)
    e = env(ds)
    assert e["DP_ENFORCE_MEMORY_UNITS"] == "true" and e["DP_REPLICA_HBM_SHARE"] == "true"
    assert e["DP_PRESTART_HEALTH_CHECK"] == "true"
    vols = {v["name"]: v for v in ds["spec"]["template"]["spec"]["volumes"]}
    (dp,) = [m for m in container(ds)["volumeMounts"] if m["mountPath"] == "/var/lib/kubelet/device-plugins"]
    assert vols[dp["name"]]["hostPath"]["path"] == dp["mountPath"]
    off = env(daemonset())
    assert off["DP_ENFORCE_MEMORY_UNITS"] == "false" and off["DP_PRESTART_HEALTH_CHECK"] == "false"
    assert off["DP_CONTAINER_HBM_METRICS"] == "true" and off["DP_MEMCAP_LD_SO_PRELOAD"] == "false"
    assert env(daemonset({"memcapLdSoPreload": True}))["DP_MEMCAP_LD_SO_PRELOAD"] == "true"
    assert env(daemonset({"containerHbmMetrics": False}))["DP_CONTAINER_HBM_METRICS"] == "false"


def test_metrics_and_node_feature_labels():
    ds = daemonset({"metrics": {"enabled": True, "port": 9500}, "nodeFeatureLabels": {"enabled": True}})
    check_consistent(ds)
    c = container(ds)
    # bound to the pod's own IP (downward API), not every interface
    # the pod IP for Prometheus, loopback for kubectl port-forward and in-pod tools
    assert env(ds)["DP_METRICS_ADDR"] == "$(POD_IP):9500,127.0.0.1:9500" and env(ds)["DP_NODE_LABELS_FILE"]
    pod_ip = [e for e in c["env"] if e["name"] == "POD_IP"][0]
    assert pod_ip["valueFrom"] == {"fieldRef": {"fieldPath": "status.podIP"}}
    names = [e["name"] for e in c["env"]]
    assert names.index("POD_IP") < names.index("DP_METRICS_ADDR")  # $(VAR) expands only earlier vars
    wide = daemonset({"metrics": {"enabled": True, "bindAddress": "0.0.0.0"}})
    assert env(wide)["DP_METRICS_ADDR"] == "0.0.0.0:9400"
    assert c["ports"] == [{"name": "metrics", "containerPort": 9500, "protocol": "TCP"}]
    assert c["livenessProbe"]["httpGet"] == {"path": "/healthz", "port": "metrics"}
    ann = ds["spec"]["template"]["metadata"]["annotations"]
    assert ann["prometheus.io/scrape"] == "true" and ann["prometheus.io/port"] == "9500"
    vols = {v["name"] for v in ds["spec"]["template"]["spec"]["volumes"]}
    assert {"pod-resources", "nfd-features"} <= vols


def test_reference_value_names_win():
    """A reference values file: migStrategy / nvidiaDriverRoot, compatWithCPUManager."""
    ds = daemonset({"migStrategy": "mixed", "nvidiaDriverRoot": "/run/amd", "compatWithCPUManager": True,
                    "passDeviceSpecs": False})
    check_consistent(ds)
    e = env(ds)
    assert e["PARTITION_STRATEGY"] == "mixed" and e["DRIVER_ROOT"] == "/run/amd"
    assert e["PASS_DEVICE_SPECS"] == "true"  # compat mode always passes device specs
    assert container(ds)["securityContext"] == {"privileged": True, "readOnlyRootFilesystem": True}


def test_legacy_api_and_overrides():
    ds = daemonset({"legacyDaemonsetAPI": True, "fullnameOverride": "gpu-plugin",
                    "image": {"tag": "v9"}, "devices": "0,1", "disableHealthChecks": "all",
                    "extraEnv": [{"name": "ADP_LOG_LEVEL", "value": "debug"}],
                    "selectorLabelsOverride": {"app": "gpu"}, "runtimeClassName": "amd"})
    check_consistent(ds)
    assert ds["apiVersion"] == "extensions/v1beta1" and "selector" not in ds["spec"]
    assert ds["metadata"]["name"] == "gpu-plugin"
    assert container(ds)["image"] == "amdgpu-device-plugin:v9"
    e = env(ds)
    assert e["AMD_DP_DEVICES"] == "0,1" and e["DP_DISABLE_HEALTHCHECKS"] == "all" and e["ADP_LOG_LEVEL"] == "debug"
    assert ds["spec"]["template"]["metadata"]["labels"] == {"app": "gpu"}
    assert ds["spec"]["template"]["spec"]["runtimeClassName"] == "amd"


@pytest.mark.parametrize("strategy", ["none", "single", "mixed"])
def test_partition_strategies(strategy):
    ds = daemonset({"partitionStrategy": strategy, "resourceConfig": "", "replicaCuMask": True})
    check_consistent(ds)
    assert env(ds)["PARTITION_STRATEGY"] == strategy
    assert "RESOURCE_CONFIG" not in env(ds) and env(ds)["REPLICA_CU_MASK"] == "true"
    assert env(ds)["DP_MEMORY_UNIT_CU_SLOTS"] == "proportional"


@pytest.mark.parametrize("values,policy,unit", [({}, "auto", "auto"),
                                                ({"replicaPolicy": "spread", "autoReplicaUnit": "cu-slot"},
                                                 "spread", "cu-slot"),
                                                ({"replicaPolicy": None, "autoReplicaUnit": None}, "auto", "auto")])
def test_replica_policy_and_unit_values(values, policy, unit):
    ds = daemonset(values)
    check_consistent(ds)
    assert env(ds)["REPLICA_POLICY"] == policy and env(ds)["AUTO_REPLICA_UNIT"] == unit


def test_memory_unit_cu_slots_value():
    ds = daemonset({"replicaCuMask": True, "memoryUnitCuSlots": "whole"})
    check_consistent(ds)
    assert env(ds)["DP_MEMORY_UNIT_CU_SLOTS"] == "whole" and env(ds)["REPLICA_CU_MASK"] == "true"


def test_renderer_trims_and_pipes_like_go_templates():
    r = helm_render.Renderer({"a": {"b": ""}, "n": 0, "s": "x+y"}, {}, {"Name": "rel"})
    nodes = r.load('{{- define "t" -}} [{{ . | quote }}] {{- end }}'
                   'A {{- .Values.a.b | default "d" | quote }} {{ include "t" "v" }}\n'
                   '{{- if .Values.n }}no{{ else if .Values.s }} {{ .Values.s | replace "+" "_" }}{{ end }}'
                   '{{ $x := printf "%s-%s" .Release.Name "c" }}{{ $x | trunc 4 }}{{/* c */}}')
    assert r.render_nodes(nodes, r.root, {}) == 'A"d" ["v"] x_yrel-'


def test_prometheus_operator_objects():
    """metrics.serviceMonitor / metrics.prometheusRule: a headless Service over
    the pods' metrics port, a ServiceMonitor selecting it, and alert rules whose
    metrics the daemon exports; nothing without metrics.enabled."""
    import glob
    import re
    vals = {"metrics": {"enabled": True, "port": 9500, "serviceMonitor": {"enabled": True, "labels": {"release": "kp"}},
                        "prometheusRule": {"enabled": True, "hbmGrantRatio": 0.9}}}
    out = helm_render.render(vals)
    svc, sm = [d for d in yaml.safe_load_all(out["servicemonitor.yaml"]) if d]
    (rule,) = [d for d in yaml.safe_load_all(out["prometheusrule.yaml"]) if d]
    ds = daemonset(vals)
    pod_labels = ds["spec"]["template"]["metadata"]["labels"]
    assert svc["kind"] == "Service" and svc["spec"]["clusterIP"] == "None"
    assert svc["spec"]["selector"].items() <= pod_labels.items()
    (port,) = svc["spec"]["ports"]
    assert port["port"] == 9500 and port["targetPort"] == "metrics"
    assert {p["name"] for p in container(ds)["ports"]} == {"metrics"}
    assert sm["kind"] == "ServiceMonitor" and sm["metadata"]["labels"]["release"] == "kp"
    assert sm["spec"]["selector"]["matchLabels"].items() <= svc["metadata"]["labels"].items()
    assert sm["spec"]["endpoints"] == [{"port": "metrics", "path": "/metrics", "interval": "30s"}]
    rules = rule["spec"]["groups"][0]["rules"]
    assert len(rules) == 19 and all(r["alert"].startswith("AmdGpu") for r in rules)
    over = [r for r in rules if r["alert"] == "AmdGpuContainerOverHbmGrant"][0]
    assert "amdgpu_dp_container_hbm_over_grant" in over["expr"] and over["labels"]["severity"] == "critical"
    assert "> 0.9" in [r for r in rules if r["alert"] == "AmdGpuContainerNearHbmGrant"][0]["expr"]
    # every metric an alert uses is one the daemon exports
    src = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "native", "src", "*", "*.cc")))
    for r in rules:
        for name in re.findall(r"amdgpu_dp_\w+", r["expr"]):
            assert f'"{name}' in src or f"{name} " in src or f"{name}{{" in src, name
    off = helm_render.render({"metrics": {"enabled": False, "serviceMonitor": {"enabled": True},
                                          "prometheusRule": {"enabled": True}}})
    assert not off["servicemonitor.yaml"].strip() and not off["prometheusrule.yaml"].strip()


def test_grafana_dashboard_configmap():
    """metrics.grafanaDashboard: a ConfigMap with the sidecar's label holding the
    dashboard JSON; every metric a panel queries is one the daemon exports."""
    import glob
    import json
    import re
    out = helm_render.render({"metrics": {"enabled": True, "grafanaDashboard": {"enabled": True}}})
    (cm,) = [d for d in yaml.safe_load_all(out["grafana-dashboard.yaml"]) if d]
    assert cm["kind"] == "ConfigMap" and cm["metadata"]["labels"]["grafana_dashboard"] == "1"
    assert cm["metadata"]["namespace"] == daemonset({})["metadata"]["namespace"]
    dash = json.loads(cm["data"]["amdgpu-device-plugin.json"])
    with open(os.path.join(helm_render.CHART, "dashboards", "amdgpu-device-plugin.json")) as f:
        assert dash == json.load(f)
    assert dash["uid"] == "amdgpu-device-plugin" and len(dash["panels"]) >= 8
    ids = [p["id"] for p in dash["panels"]]
    assert len(ids) == len(set(ids))
    src = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "native", "src", "*", "*.cc")))
    exprs = [t["expr"] for p in dash["panels"] for t in p["targets"]]
    names = {n for e in exprs for n in re.findall(r"amdgpu_dp_\w+", e)}
    assert "amdgpu_dp_rpc_residency_seconds_bucket" in names
    for name in names:
        base = re.sub(r"_(bucket|sum|count)$", "", name)
        assert f'"{base}' in src or f"{base} " in src or f"{base}{{" in src, name
    # the sidecar may watch another namespace
    other = helm_render.render({"metrics": {"enabled": True,
                                            "grafanaDashboard": {"enabled": True, "namespace": "monitoring"}}})
    assert yaml.safe_load(other["grafana-dashboard.yaml"])["metadata"]["namespace"] == "monitoring"
    assert not helm_render.render({"metrics": {"enabled": True}})["grafana-dashboard.yaml"].strip()
    assert not helm_render.render({"metrics": {"enabled": False, "grafanaDashboard": {"enabled": True}}})[
        "grafana-dashboard.yaml"].strip()


@pytest.mark.parametrize("strategy,mounted", [("envvar", False), ("volume-mounts", False),
                                               ("cdi-annotations", True), ("cdi-cri", True)])
def test_cdi_strategies_write_the_spec_where_the_runtime_reads_it(strategy, mounted):
    """The CDI list strategies make the daemon write a CDI spec (--cdi-spec-dir,
    /var/run/cdi): the chart mounts the host's /var/run/cdi there, so the
    container runtime sees it -- and the read-only root filesystem is never
    written."""
    ds = daemonset({"deviceListStrategy": strategy})
    check_consistent(ds)
    mounts = {m["name"]: m for m in container(ds)["volumeMounts"]}
    vols = {v["name"]: v for v in ds["spec"]["template"]["spec"]["volumes"]}
    assert ("cdi-specs" in mounts) == mounted
    if mounted:
        assert mounts["cdi-specs"]["mountPath"] == "/var/run/cdi"
        assert vols["cdi-specs"]["hostPath"] == {"path": "/var/run/cdi", "type": "DirectoryOrCreate"}


def test_metrics_network_policy():
    """metrics.networkPolicy: only the listed peers reach the metrics port (the
    endpoints are unauthenticated); off by default and without metrics."""
    out = helm_render.render({"metrics": {"enabled": True, "networkPolicy": {"enabled": True}}})
    (np,) = [d for d in yaml.safe_load_all(out["networkpolicy.yaml"]) if d]
    assert np["kind"] == "NetworkPolicy" and np["spec"]["policyTypes"] == ["Ingress"]
    ds = daemonset({"metrics": {"enabled": True}})
    assert np["spec"]["podSelector"]["matchLabels"].items() <= ds["spec"]["template"]["metadata"]["labels"].items()
    (rule,) = np["spec"]["ingress"]
    assert rule["ports"] == [{"port": 9400, "protocol": "TCP"}]
    assert rule["from"] == [{"namespaceSelector": {"matchLabels": {"kubernetes.io/metadata.name": "monitoring"}}}]
    custom = helm_render.render({"metrics": {"enabled": True, "port": 9500, "networkPolicy": {
        "enabled": True, "from": [{"podSelector": {"matchLabels": {"app": "prometheus"}}}]}}})
    (np2,) = [d for d in yaml.safe_load_all(custom["networkpolicy.yaml"]) if d]
    assert np2["spec"]["ingress"][0] == {"ports": [{"port": 9500, "protocol": "TCP"}],
                                         "from": [{"podSelector": {"matchLabels": {"app": "prometheus"}}}]}
    for vals in ({}, {"metrics": {"enabled": True}}, {"metrics": {"enabled": False, "networkPolicy": {"enabled": True}}}):
        assert not helm_render.render(vals)["networkpolicy.yaml"].strip()


@pytest.mark.parametrize("values,want", [
    ({}, "gpu:gpu-mem-gb:-1"),                                           # MiB units: the name is right
    ({"replicaCuMask": True}, "gpu:gpu-slot:-1"),                        # auto -> CU slots: renamed
    ({"autoReplicaUnit": "cu-slot"}, "gpu:gpu-slot:-1"),
    ({"replicaCuMask": True, "autoReplicaUnit": "mib"}, "gpu:gpu-mem-gb:-1"),
    ({"replicaCuMask": True, "resourceConfig": "gpu:mem-slots:-1"}, "gpu:mem-slots:-1"),  # the user's own name
])
def test_cu_slot_units_do_not_keep_a_gigabyte_name(values, want):
    """A memory unit that is a CU slot (~9 GiB on an MI355X) under the default
    resource name gpu-mem-gb would let a pod asking for 16 "GB" take half the
    GPU: with CU-slot units the chart's default renders as gpu-slot instead;
    MiB units and a name the user chose are left alone."""
    ds = daemonset(values)
    check_consistent(ds)
    assert env(ds)["RESOURCE_CONFIG"] == want


@pytest.mark.parametrize("values,hold,limit,window", [
    ({}, "120000", "3", "600000"),
    ({"resetRecoveryHoldMs": 0, "resetFlap": {"limit": 0, "windowMs": 60000}}, "0", "0", "60000"),
])
def test_reset_recovery_and_flap_values(values, hold, limit, window):
    """The event-gap hold and the reset-flap damping reach the daemon; 0 (off)
    survives the template (no `default` turning it back on)."""
    ds = daemonset(values)
    check_consistent(ds)
    e = env(ds)
    assert (e["DP_RESET_RECOVERY_HOLD_MS"], e["DP_RESET_FLAP_LIMIT"], e["DP_RESET_FLAP_WINDOW_MS"]) == \
        (hold, limit, window)


def test_defer_layout_changes_value_mounts_pod_resources():
    """deferLayoutChanges reaches the daemon and mounts the kubelet's
    PodResources socket (which IDs running pods hold) even without metrics."""
    e = env(daemonset())
    assert e["DP_DEFER_LAYOUT_CHANGES"] == "false"
    ds = daemonset({"deferLayoutChanges": True})
    check_consistent(ds)
    assert env(ds)["DP_DEFER_LAYOUT_CHANGES"] == "true"
    mounts = {m["name"]: m for m in container(ds)["volumeMounts"]}
    assert mounts["pod-resources"]["readOnly"] is True
    assert any(v["name"] == "pod-resources" for v in ds["spec"]["template"]["spec"]["volumes"])
    ds0 = daemonset()
    assert "pod-resources" not in {m["name"] for m in container(ds0)["volumeMounts"]}


def test_extra_event_types_reach_both_containers():
    """healthEventExtraTypes: the plugin counts them and the relay registers
    them (each reads DP_HEALTH_EVENT_EXTRA_TYPES); unset by default."""
    ds = daemonset({"healthEventExtraTypes": "12,13"})
    assert env(ds)["DP_HEALTH_EVENT_EXTRA_TYPES"] == "12,13"
    r = relay(ds)
    assert {e["name"]: e.get("value") for e in r["env"]}["DP_HEALTH_EVENT_EXTRA_TYPES"] == "12,13"
    ds = daemonset()
    assert "DP_HEALTH_EVENT_EXTRA_TYPES" not in env(ds)
    assert "DP_HEALTH_EVENT_EXTRA_TYPES" not in {e["name"] for e in relay(ds)["env"]}

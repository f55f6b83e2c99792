"""Packaging consistency: helm values/templates, static manifests, example pods.

Every environment variable a manifest sets must be one the daemon reads (its
--help lists them), and the helm values keep the reference chart's key names
(reference deployments/helm/nvidia-device-plugin/values.yaml:1-47) where the
meaning carries over.
"""

import glob
import os
import re
import subprocess

import yaml

from k8s_gpu_sharing_plugin_amd import DAEMON

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHART = os.path.join(ROOT, "deployments", "helm", "amd-gpu-device-plugin")
# POD_IP: downward-API value the kubelet expands into DP_METRICS_ADDR
KNOWN_EXTRA_ENV = {"DP_DISABLE_HEALTHCHECKS", "DP_HEALTH_POLL_MS", "DP_MAX_RETIRED_PAGES", "POD_IP"}


def daemon_envs():
    out = subprocess.run([DAEMON, "--help"], capture_output=True, text=True, timeout=10).stdout
    return set(re.findall(r"\(env ([A-Z_]+)", out)) | KNOWN_EXTRA_ENV


def test_helm_values_keep_compatible_keys():
    with open(os.path.join(CHART, "values.yaml")) as f:
        v = yaml.safe_load(f)
    for key in ("legacyDaemonsetAPI", "compatWithCPUManager", "failOnInitError", "deviceListStrategy",
                "deviceIDStrategy", "resourceConfig", "nameOverride", "fullnameOverride",
                "selectorLabelsOverride", "namespace", "image", "updateStrategy", "podSecurityContext",
                "securityContext", "resources", "nodeSelector", "affinity", "tolerations", "runtimeClassName"):
        assert key in v, key
    assert v["partitionStrategy"] == "none"  # replaces migStrategy
    assert v["driverRoot"] == "/"            # replaces nvidiaDriverRoot
    assert v["resourceConfig"] == "gpu:gpu-mem-gb:-1"
    assert v["nodeSelector"] == {"gpushare": "true"}
    assert {"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"} in v["tolerations"]


def test_helm_template_envs_are_daemon_envs():
    with open(os.path.join(CHART, "templates", "daemonset.yaml")) as f:
        text = f.read()
    names = set(re.findall(r"name: ([A-Z][A-Z_]+)", text))
    assert names and names <= daemon_envs(), names - daemon_envs()
    assert "system-node-critical" in text
    assert "/var/lib/kubelet/device-plugins" in text


def test_static_manifests():
    files = glob.glob(os.path.join(ROOT, "deployments", "static", "*.yml")) + [
        os.path.join(ROOT, "amd-gpu-device-plugin.yml")]
    assert len(files) >= 4
    envs = daemon_envs()
    for path in files:
        with open(path) as f:
            doc = yaml.safe_load(f)
        assert doc["kind"] == "DaemonSet"
        spec = doc["spec"]["template"]["spec"]
        c = spec["containers"][0]
        for e in c["env"]:
            assert e["name"] in envs, (path, e["name"])
        mounts = {m["mountPath"] for m in c["volumeMounts"]}
        assert "/var/lib/kubelet/device-plugins" in mounts
        assert spec["priorityClassName"] == "system-node-critical"
        if "extensions-v1beta1" in path:
            assert doc["apiVersion"] == "extensions/v1beta1"
        else:
            assert doc["apiVersion"] == "apps/v1"
            assert doc["spec"]["selector"]["matchLabels"] == doc["spec"]["template"]["metadata"]["labels"]
        if "cpumanager" in path:
            assert c["securityContext"] == {"privileged": True, "readOnlyRootFilesystem": True}
        else:  # the plugin container itself never runs privileged, and writes only to its volumes
            assert c["securityContext"]["capabilities"]["drop"] == ["ALL"], path
            assert c["securityContext"]["readOnlyRootFilesystem"] is True, path
        vols = {v["name"] for v in spec["volumes"]}
        for ctr in spec["containers"]:
            assert {m["name"] for m in ctr["volumeMounts"]} <= vols, (path, ctr["name"])
        if "health-events" in path:
            # privilege separation: only the relay is privileged, and the two share the socket dir
            (relay,) = [x for x in spec["containers"] if x["name"] == "event-relay"]
            assert relay["securityContext"] == {"privileged": True, "readOnlyRootFilesystem": True}
            assert relay["args"] == ["--event-relay", "--health-event-socket", "/run/amdgpu-dp-events/events.sock"]
            assert {e["name"]: e["value"] for e in c["env"]}["DP_HEALTH_EVENT_SOCKET"] == \
                "/run/amdgpu-dp-events/events.sock"


def test_example_pods_request_amd_resources():
    seen = set()
    for path in glob.glob(os.path.join(ROOT, "examples", "pods", "*.yml")):
        with open(path) as f:
            pod = yaml.safe_load(f)
        assert pod["kind"] == "Pod"
        for c in pod["spec"]["containers"]:
            limits = (c.get("resources") or {}).get("limits") or {}
            for r in limits:
                assert r.startswith("amd.com/"), (path, r)
                seen.add(r)
    assert {"amd.com/gpu", "amd.com/sharedgpu", "amd.com/gpu-mem-gb", "amd.com/cpx-1xcd.36gb"} <= seen


def test_release_versions_agree():
    """RELEASE.md step 1: every place that carries the version says the same."""
    import glob
    import re
    import k8s_gpu_sharing_plugin_amd as pkg
    root = pkg.REPO_ROOT

    def read(p):
        with open(os.path.join(root, p)) as f:
            return f.read()
    version = re.search(r"^VERSION\s*\?=\s*(\S+)", read("versions.mk"), re.M).group(1)
    assert pkg.__version__ == version
    assert f'set(ADP_VERSION "{version}"' in read("native/CMakeLists.txt")
    chart = read("deployments/helm/amd-gpu-device-plugin/Chart.yaml")
    assert f'version: "{version}"' in chart and f'appVersion: "{version}"' in chart
    for m in ["amd-gpu-device-plugin.yml", *glob.glob(os.path.join(root, "deployments/static/*.yml"))]:
        assert f"amdgpu-device-plugin:{version}" in read(m), m
    for d in ("ubuntu", "ubi9"):
        assert "ENTRYPOINT" in read(f"deployments/container/Dockerfile.{d}")


def test_helm_template_accepts_reference_value_names():
    """A reference values file (values.yaml:3,7 migStrategy / nvidiaDriverRoot)
    keeps working: the template prefers those names when they are set."""
    with open(os.path.join(CHART, "templates", "daemonset.yaml")) as f:
        text = f.read()
    assert "coalesce .Values.migStrategy .Values.partitionStrategy" in text
    assert "coalesce .Values.nvidiaDriverRoot .Values.driverRoot" in text


def test_dev_image_and_docker_targets():
    """B02: the development image carries the build/test toolchain, and every
    docker-<target> rule runs `make <target>` in it (reference Makefile:44-74)."""
    text = open(os.path.join(ROOT, "docker", "Dockerfile.devel")).read()
    for pkg in ("cmake", "ninja-build", "libnghttp2-dev", "libyaml-dev", "amd-smi-lib", "pytest", "grpcio"):
        assert pkg in text, pkg
    for target in ("build", "test", "lint", "asan", "tsan", "coverage"):
        r = subprocess.run(["make", "-n", f"docker-{target}", "SKIP_IMAGE_BUILD=1", "DOCKER=docker"], cwd=ROOT,
                           capture_output=True, text=True, timeout=30)
        assert r.returncode == 0, r.stderr
        run = [ln for ln in r.stdout.splitlines() if "docker run" in ln or "make " + target in ln]
        assert run and run[-1].rstrip().endswith(f"make {target}"), r.stdout

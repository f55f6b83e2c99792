"""Container images: every library a shipped binary needs is in the image.

Static check of each runtime stage of deployments/container/Dockerfile.*: the
ELF files the stage ships (the daemon and probe built here, the ROCm libraries
it COPYs from /opt/rocm/lib of this same image) are read with readelf, their
DT_NEEDED entries and their dlopen targets are collected, and each soname must
be provided by the base image, an installed package, or a COPY'd file.

Round 1 shipped libamd_smi without libdrm_amdgpu (which it dlopens) and the
probe without the HIP runtime's needed libraries; no container runtime exists
here, so this is the guard (each stage also re-checks with ldd at build time).

Parity: the reference builds its image in CI (.gitlab-ci.yml:82-105) from
deployments/container/Dockerfile.ubuntu:15-55, which needs only the Go binary.
"""

import glob
import os
import re
import subprocess

import pytest

from k8s_gpu_sharing_plugin_amd import DAEMON, PROBE_BIN
from k8s_gpu_sharing_plugin_amd.utils import image

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM_LIB = "/opt/rocm/lib"
# The Dockerfile model shared with the rootfs assembly (tests/test_image_rootfs.py).
BASE, PACKAGES, BUILT, stages = image.BASE, image.PACKAGES, image.BUILT, image.stages
# Libraries the daemon itself dlopens (native/src/smi/smi.cc, native/src/daemon/yaml.cc).
DAEMON_DLOPENS = {"libamd_smi.so.26", "libyaml-0.so.2"}


def stage_contents(lines):
    pkgs, copies, _, _ = image.stage_contents(lines)
    return pkgs, [src for sources, _ in copies for src in sources]


def sonames(path):
    out = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
    return set(re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", out))


def dlopen_targets(path):
    """Library names an ELF carries as strings (what it may dlopen)."""
    out = subprocess.run(["strings", path], capture_output=True, text=True, check=True).stdout
    return {s for s in out.split() if re.fullmatch(r"lib[a-z_0-9-]+\.so(\.[0-9]+)+", s)}


def runtime_stages():
    for df in sorted(glob.glob(os.path.join(REPO, "deployments", "container", "Dockerfile.*"))):
        dist = df.rsplit(".", 1)[1]
        for name, base, lines in stages(df):
            if name == "build":
                continue
            yield pytest.param(dist, name, base, lines, id=f"{dist}-{name}")


@pytest.mark.parametrize("dist,name,base,lines", list(runtime_stages()))
def test_runtime_stage_provides_every_needed_library(dist, name, base, lines):
    if not (os.path.exists(DAEMON) and os.path.exists(PROBE_BIN)):
        pytest.skip("native artefacts not built")
    image.ensure_image_tree()
    pkgs, copies = stage_contents(lines)
    shipped, copied_names = [], set()
    for src in copies:
        if src in BUILT:
            shipped.append(BUILT[src])
            continue
        assert src.startswith(ROCM_LIB + "/"), f"{dist}/{name}: unexpected COPY source {src}"
        files = glob.glob(src)
        assert files, f"{dist}/{name}: COPY {src} matches nothing in this ROCm install"
        copied_names |= {os.path.basename(f) for f in files}
        shipped += [f for f in files if not os.path.islink(f)]
    assert shipped, f"{dist}/{name} ships nothing"
    provided = set(BASE[dist]) | copied_names
    provided |= {so for so, pkg in PACKAGES[dist].items() if pkg in pkgs}
    need = {}
    for f in shipped:
        for so in sonames(f):
            need.setdefault(so, set()).add(os.path.basename(f))
        if os.path.basename(f) == "amdgpu-device-plugin":
            for so in DAEMON_DLOPENS:
                need.setdefault(so, set()).add("amdgpu-device-plugin (dlopen)")
        elif f.startswith(ROCM_LIB):
            own = os.path.basename(f).split(".so")[0]
            for so in dlopen_targets(f):
                if so.split(".so")[0] != own and so not in ("libamdhip64.so",):
                    need.setdefault(so, set()).add(os.path.basename(f) + " (dlopen)")
    missing = {so: sorted(by) for so, by in need.items() if so not in provided}
    assert not missing, f"{dist}/{name} (FROM {base}) lacks {missing}; packages {sorted(pkgs)}"


def test_dockerfile_ldd_checks_and_targets():
    ub = open(os.path.join(REPO, "deployments", "container", "Dockerfile.ubuntu")).read()
    names = [s[0] for s in stages(os.path.join(REPO, "deployments", "container", "Dockerfile.ubuntu"))]
    assert names[-1] == "runtime" and "validation" in names  # default target = the DaemonSet image
    assert ub.count('grep "not found"') == 2
    ubi = open(os.path.join(REPO, "deployments", "container", "Dockerfile.ubi9")).read()
    assert 'grep "not found"' in ubi
    pod = open(os.path.join(REPO, "examples", "pods", "pod-validate.yml")).read()
    assert "amdgpu-device-plugin-validation" in pod


def test_daemon_dlopen_list_matches_the_source():
    smi = open(os.path.join(REPO, "native", "src", "smi", "smi.cc")).read()
    yml = open(os.path.join(REPO, "native", "src", "daemon", "yaml.cc")).read()
    assert '"libamd_smi.so.26"' in smi and '"libyaml-0.so.2"' in yml

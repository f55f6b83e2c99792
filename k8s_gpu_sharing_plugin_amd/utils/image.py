"""The container images without a container engine.

No docker/buildah exists here, so the images' runtime stages are checked two
ways:

* statically (tests/test_image_deps.py): every DT_NEEDED and dlopen target of
  what a stage ships is provided by its base image, a package or a COPY;
* by assembling the stage's root filesystem (``build_rootfs``) from the same
  parts -- the base image's glibc/C++ runtime and the stage's apt packages
  taken from this Ubuntu 22.04 host (the base is ubuntu:22.04), the stage's
  COPY sources from this tree and /opt/rocm -- and running the daemon in it
  with ``unshare -r chroot`` (tests/test_image_rootfs.py). Only what the
  Dockerfile puts in the image is in that tree, so a library the stage forgot
  fails the run as it would fail the real image.

Parity: the reference builds its image in CI from
/root/reference/deployments/container/Dockerfile.ubuntu:15-55.
"""

import glob
import json
import os
import re
import shlex
import shutil
import subprocess

from .. import PROBE_BIN, REPO_ROOT

ROCM_LIB = "/opt/rocm/lib"
HOST_LIB = "/lib/x86_64-linux-gnu"

# Libraries every base image has (glibc + the C++ runtime apt/microdnf use).
BASE = {
    "ubuntu": {"libc.so.6", "libm.so.6", "ld-linux-x86-64.so.2", "libpthread.so.0", "libdl.so.2", "librt.so.1",
               "libgcc_s.so.1", "libstdc++.so.6", "libz.so.1", "libzstd.so.1"},
    "ubi9": {"libc.so.6", "libm.so.6", "ld-linux-x86-64.so.2", "libpthread.so.0", "libdl.so.2", "librt.so.1",
             "libgcc_s.so.1", "libz.so.1", "libzstd.so.1"},
}
# soname -> package that installs it, per distribution.
PACKAGES = {
    "ubuntu": {"libnghttp2.so.14": "libnghttp2-14", "libdrm.so.2": "libdrm2", "libdrm_amdgpu.so.1": "libdrm-amdgpu1",
               "libyaml-0.so.2": "libyaml-0-2", "libelf.so.1": "libelf1", "libnuma.so.1": "libnuma1",
               "libz.so.1": "zlib1g", "libzstd.so.1": "libzstd1", "libstdc++.so.6": "libstdc++6"},
    "ubi9": {"libnghttp2.so.14": "libnghttp2", "libdrm.so.2": "libdrm", "libdrm_amdgpu.so.1": "libdrm",
             "libyaml-0.so.2": "libyaml", "libelf.so.1": "elfutils-libelf", "libnuma.so.1": "numactl-libs",
             "libstdc++.so.6": "libstdc++"},
}
# The build stage's outputs, as built in this tree: the daemon and the shim of
# build/image (the stage's cmake line: ADP_TEST_HOOKS=OFF), the probe.
IMAGE_DIR = os.path.join(REPO_ROOT, "build", "image")
IMAGE_DAEMON = os.path.join(IMAGE_DIR, "amdgpu-device-plugin")
BUILT = {"/build/amdgpu-device-plugin": IMAGE_DAEMON, "/build/amdgpu-dp-probe": PROBE_BIN,
         "/build/libadp_memcap.so": os.path.join(IMAGE_DIR, "libadp_memcap.so")}


def ensure_image_tree():
    """build/image, built here on first use (it travels to the GPU box built)."""
    if not all(os.path.exists(BUILT[k]) for k in ("/build/amdgpu-device-plugin", "/build/libadp_memcap.so")):
        from . import build
        build.build_image_tree()


def dockerfile(dist="ubuntu"):
    return os.path.join(REPO_ROOT, "deployments", "container", f"Dockerfile.{dist}")


def stages(path):
    """[(name, base image, [instruction lines])] of a Dockerfile (continuations joined)."""
    text = open(path).read().replace("\\\n", " ")
    out = []
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        m = re.match(r"FROM\s+(\S+)(?:\s+AS\s+(\S+))?", line, re.I)
        if m:
            out.append((m.group(2) or "", m.group(1), []))
        elif out:
            out[-1][2].append(line)
    return out


def stage_contents(lines):
    """(apt/microdnf packages, [(COPY --from=build sources, destination)], ld.so.conf.d lines, entrypoint)."""
    pkgs, copies, ldconf, entry = set(), [], [], None
    for line in lines:
        if line.startswith("RUN"):
            for cmd in re.split(r"&&|;", line[3:]):
                words = shlex.split(cmd)
                if words[:2] in (["apt-get", "install"], ["microdnf", "install"]):
                    pkgs |= {w for w in words[2:] if not w.startswith("-")}
                m = re.match(r"\s*echo\s+(\S+)\s*>\s*(/etc/ld\.so\.conf\.d/\S+)", cmd)
                if m:
                    ldconf.append((m.group(2), m.group(1)))
        elif line.startswith("COPY") and "--from=build" in line:
            args = [a for a in shlex.split(line)[1:] if not a.startswith("--")]
            copies.append((args[:-1], args[-1]))
        elif line.startswith("ENTRYPOINT"):
            entry = json.loads(line[len("ENTRYPOINT"):].strip())
    return pkgs, copies, ldconf, entry


def _host_file(soname):
    for d in (HOST_LIB, "/usr/lib/x86_64-linux-gnu", "/lib64"):
        p = os.path.join(d, soname)
        if os.path.exists(p):
            return os.path.realpath(p)
    return None


def _put(src, dest_dir, name=None):
    os.makedirs(dest_dir, exist_ok=True)
    dst = os.path.join(dest_dir, name or os.path.basename(src))
    if os.path.islink(src) and name is None:
        if os.path.lexists(dst):
            os.unlink(dst)
        os.symlink(os.readlink(src), dst)
    else:
        shutil.copy2(os.path.realpath(src), dst)
    return dst


def build_rootfs(dest, dist="ubuntu", stage="runtime"):
    """Assembles `stage` of Dockerfile.<dist> under `dest` and returns a
    manifest: what came from where, and package files this host lacks (an
    image built from the registry would have them; the run here goes without).
    Only ubuntu stages can be assembled from this host."""
    if dist != "ubuntu":
        raise ValueError("only the ubuntu stages can be assembled on this (Ubuntu 22.04) host")
    ensure_image_tree()
    (name, base, lines), = [s for s in stages(dockerfile(dist)) if s[0] == stage]
    pkgs, copies, ldconf, entry = stage_contents(lines)
    if os.path.exists(dest):
        shutil.rmtree(dest)
    for d in ("usr/bin", "lib64", "etc/ld.so.conf.d", "tmp", "dev", "sys", "proc", "run", "var/lib"):
        os.makedirs(os.path.join(dest, d), exist_ok=True)
    libdir = os.path.join(dest, HOST_LIB.lstrip("/"))
    manifest = {"dockerfile": os.path.relpath(dockerfile(dist), REPO_ROOT), "stage": stage, "base": base,
                "base_libs": [], "packages": {}, "missing_package_files": [], "copied": [], "entrypoint": entry}
    # the base image: glibc and the C++ runtime, as ubuntu:22.04 has them
    for so in sorted(BASE[dist]):
        src = _host_file(so)
        if not src:
            manifest["missing_package_files"].append(so)
            continue
        if so == "ld-linux-x86-64.so.2":
            _put(src, os.path.join(dest, "lib64"), so)
        _put(src, libdir, so)
        manifest["base_libs"].append(so)
    # the stage's packages (their shared libraries)
    for pkg in sorted(pkgs):
        for so in [s for s, p in PACKAGES[dist].items() if p == pkg]:
            src = _host_file(so)
            if src:
                _put(src, libdir, so)
                manifest["packages"].setdefault(pkg, []).append(so)
            else:
                manifest["missing_package_files"].append(f"{pkg}:{so}")
    # COPY --from=build
    for sources, dst in copies:
        for src in sources:
            if src in BUILT:
                files = [BUILT[src]]
            else:
                files = sorted(glob.glob(src))
            for f in files:
                target_dir = os.path.join(dest, dst.lstrip("/")) if dst.endswith("/") else \
                    os.path.join(dest, os.path.dirname(dst).lstrip("/"))
                nm = None if dst.endswith("/") else os.path.basename(dst)
                _put(f, target_dir, nm)
                manifest["copied"].append(f"{f} -> {dst if nm else os.path.join(dst, os.path.basename(f))}")
    for path, line in ldconf:
        with open(os.path.join(dest, path.lstrip("/")), "w") as fh:
            fh.write(line + "\n")
    with open(os.path.join(dest, "etc/ld.so.conf"), "w") as fh:
        fh.write("include /etc/ld.so.conf.d/*.conf\n" + HOST_LIB + "\n")
    subprocess.run(["ldconfig", "-r", dest], check=True, capture_output=True)
    return manifest


def chroot_cmd(rootfs, argv, binds=()):
    """argv run as root of a user namespace chrooted into `rootfs`; `binds`
    (host dirs, e.g. /dev /sys for real GPUs) are bind-mounted at the same path
    first (a mount namespace of the same unshare)."""
    if not binds:
        return ["unshare", "-r", "chroot", rootfs, *argv]
    script = " && ".join(f"mount --rbind {shlex.quote(b)} {shlex.quote(os.path.join(rootfs, b.lstrip('/')))}"
                         for b in binds)
    script += " && exec chroot " + shlex.quote(rootfs) + " " + " ".join(shlex.quote(a) for a in argv)
    return ["unshare", "-rm", "sh", "-c", script]


def unresolved(rootfs, files):
    """{file: [sonames the image's loader cannot find]} for ELF files of the image
    (the Dockerfile's `ldd ... | grep "not found"` step, run in the image)."""
    out = {}
    for f in files:
        r = subprocess.run(chroot_cmd(rootfs, ["/lib64/ld-linux-x86-64.so.2", "--list", f]), capture_output=True,
                           text=True, timeout=60)
        missing = re.findall(r"^\s*(\S+) => not found", r.stdout, re.M)
        if missing or r.returncode != 0:
            out[f] = missing or [r.stderr.strip()[-200:]]
    return out


def image_daemon(rootfs, args=(), env=None, fixture=None, binds=(), plugin_dir="/var/lib/kubelet/device-plugins",
                 loader=False, log_path=None):
    """The daemon of an assembled runtime image, as its ENTRYPOINT runs it.
    Chrooted (root of a user namespace; `binds` of /dev and /sys for real GPUs)
    or, with `loader`, through the image's own dynamic loader (hosts without
    user namespaces; `plugin_dir` is then a host path). With `fixture` the
    amdsmi mock is copied into the image's /tmp and loaded (CPU). Returns a
    started harness.Daemon whose process is the daemon itself."""
    import tempfile
    from .. import MOCK_LIB
    from . import harness
    e = {k: v for k, v in os.environ.items() if k not in ("LD_PRELOAD", "LD_LIBRARY_PATH", "AMD_SMI_LIB")}
    e.setdefault("ADP_LOG_LEVEL", "info")
    if fixture is not None:
        shutil.copy2(MOCK_LIB, os.path.join(rootfs, "tmp", "libamdsmi_mock.so"))
        with open(os.path.join(rootfs, "tmp", "fixture.json"), "w") as f:
            json.dump(fixture, f)
        mock = "/tmp/libamdsmi_mock.so" if not loader else os.path.join(rootfs, "tmp", "libamdsmi_mock.so")
        fx = "/tmp/fixture.json" if not loader else os.path.join(rootfs, "tmp", "fixture.json")
        e.update({"AMD_SMI_LIB": mock, "AMDSMI_MOCK_FIXTURE": fx})
    e.update(env or {})

    def launch(argv):  # [DAEMON, "--device-plugin-path", dir, *args] -> the image's entrypoint
        inner = ["/usr/bin/amdgpu-device-plugin", *argv[1:]]
        return loader_cmd(rootfs, inner) if loader else chroot_cmd(rootfs, inner, binds)
    d = harness.Daemon(plugin_dir, real_smi=True, args=args, launch=launch,
                       log_path=log_path or tempfile.mktemp(prefix="adp-image-", suffix=".log"))
    d.env = e
    return d.start()


def loader_cmd(rootfs, argv):
    """argv run by the image's own dynamic loader with only the image's library
    directories (for hosts without user namespaces, e.g. the GPU box): the
    image's glibc, packages and ROCm libraries are the ones loaded -- check
    with LD_DEBUG=files (`loaded_files`) -- while /dev, /sys and /proc are the
    host's, as the chart mounts them."""
    libs = ":".join(os.path.join(rootfs, d) for d in (HOST_LIB.lstrip("/"), "opt/rocm/lib",
                                                      "usr/lib/amdgpu-device-plugin"))
    return [os.path.join(rootfs, "lib64/ld-linux-x86-64.so.2"), "--inhibit-cache", "--library-path", libs,
            os.path.join(rootfs, argv[0].lstrip("/")), *argv[1:]]


def loaded_files(ld_debug_text):
    """Shared objects a run loaded, from its LD_DEBUG=files output."""
    found = set(re.findall(r"file=(/\S+) \[0\];\s+generating link map", ld_debug_text))
    found |= set(re.findall(r"calling init: (/\S+)", ld_debug_text))
    return sorted(found)

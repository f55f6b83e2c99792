"""Build the native tree (CMake + Ninja) and the HIP probe (hipcc, gfx950).

Everything is built in-tree under ``build/`` so the artefacts travel with the
repository snapshot to the GPU box.
"""

import os
import shutil
import subprocess
import sys

from .. import BUILD_DIR, PROBE_DIR, PROBE_LIB, REPO_ROOT

NATIVE_SRC = os.path.join(REPO_ROOT, "native")
PROBE_SRC = os.path.join(NATIVE_SRC, "probe", "visibility_probe.hip")
PROTO_SRC = os.path.join(REPO_ROOT, "proto", "deviceplugin", "v1beta1", "api.proto")
DESCRIPTOR = os.path.join(REPO_ROOT, "build", "api_descriptor.pb")


def _run(cmd, **kw):
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, **kw)
    if res.returncode != 0:
        sys.stderr.write(res.stdout[-8000:])
        raise RuntimeError(f"command failed ({res.returncode}): {' '.join(cmd)}")
    return res.stdout


def build_native(jobs: int = 8, build_type: str = "Release", build_dir: str = BUILD_DIR,
                 extra_cmake=None, targets=None) -> str:
    """Configure (once) and build every native target (or `targets`). Returns the build dir."""
    generator = ["-G", "Ninja"] if shutil.which("ninja") else []
    if not os.path.exists(os.path.join(build_dir, "CMakeCache.txt")):
        os.makedirs(build_dir, exist_ok=True)
        _run(["cmake", "-S", NATIVE_SRC, "-B", build_dir, f"-DCMAKE_BUILD_TYPE={build_type}",
              *generator, *(extra_cmake or [])])
    _run(["cmake", "--build", build_dir, *(["--target", *targets] if targets else []), "--", f"-j{jobs}"])
    return build_dir


# What the image stages build (deployments/container/Dockerfile.*): the daemon
# and the shim, with the fault-injection hooks compiled out.
IMAGE_BUILD_DIR = os.path.join(REPO_ROOT, "build", "image")
IMAGE_CMAKE = ["-DADP_TEST_HOOKS=OFF"]
IMAGE_TARGETS = ["amdgpu-device-plugin", "adp_memcap"]


def build_image_tree(jobs: int = 8) -> str:
    """build/image: the image stages' cmake line and targets (ADP_TEST_HOOKS=OFF)."""
    return build_native(jobs, build_dir=IMAGE_BUILD_DIR, extra_cmake=IMAGE_CMAKE, targets=IMAGE_TARGETS)


PROBE_MAIN = os.path.join(NATIVE_SRC, "probe", "probe_main.cpp")
PROBE_EXE = os.path.join(PROBE_DIR, "amdgpu-dp-probe")


def build_probe(arch: str = "gfx950") -> str:
    """Compile the HIP visibility probe: build/probe/libadp_probe.so + amdgpu-dp-probe."""
    os.makedirs(PROBE_DIR, exist_ok=True)
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    src_mtime = max(os.path.getmtime(PROBE_SRC), os.path.getmtime(PROBE_MAIN))
    fresh = all(os.path.exists(p) and os.path.getmtime(p) >= src_mtime for p in (PROBE_LIB, PROBE_EXE))
    if fresh:
        return PROBE_LIB
    _run([hipcc, f"--offload-arch={arch}", "-O3", "-std=c++17", "-fPIC", "-shared",
          "-Wall", "-o", PROBE_LIB, PROBE_SRC])
    _run([hipcc, f"--offload-arch={arch}", "-O3", "-std=c++17", "-Wall", "-o", PROBE_EXE, PROBE_SRC,
          PROBE_MAIN])
    return PROBE_LIB


MEMCAP_BENCH_SRC = os.path.join(NATIVE_SRC, "memcap", "memcap_bench.cpp")
MEMCAP_BENCH = os.path.join(PROBE_DIR, "amdgpu-dp-memcap-bench")


def build_memcap_bench() -> str:
    """HIP host program timing the allocation path with / without the HBM-cap shim."""
    os.makedirs(PROBE_DIR, exist_ok=True)
    if os.path.exists(MEMCAP_BENCH) and os.path.getmtime(MEMCAP_BENCH) >= os.path.getmtime(MEMCAP_BENCH_SRC):
        return MEMCAP_BENCH
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    _run([hipcc, "-O2", "-std=c++17", "-Wall", "-o", MEMCAP_BENCH, MEMCAP_BENCH_SRC])
    return MEMCAP_BENCH


def build_descriptor() -> str:
    """protoc --descriptor_set_out for the kubelet API (used by the grpcio stub)."""
    if os.path.exists(DESCRIPTOR) and os.path.getmtime(DESCRIPTOR) >= os.path.getmtime(PROTO_SRC):
        return DESCRIPTOR
    protoc = shutil.which("protoc")
    if protoc is None:
        import torch  # the image ships protoc next to torch's binaries
        cand = os.path.join(os.path.dirname(torch.__file__), "bin", "protoc")
        protoc = cand if os.path.exists(cand) else None
    if protoc is None:
        raise RuntimeError("protoc not found")
    os.makedirs(os.path.dirname(DESCRIPTOR), exist_ok=True)
    _run([protoc, f"--proto_path={os.path.join(REPO_ROOT, 'proto')}",
          f"--descriptor_set_out={DESCRIPTOR}", "deviceplugin/v1beta1/api.proto"])
    return DESCRIPTOR


def build_all(probe: bool = True) -> None:
    build_native()
    build_image_tree()
    build_descriptor()
    if probe:
        build_probe()
        build_memcap_bench()


if __name__ == "__main__":
    build_all(probe="--no-probe" not in sys.argv)
    print("built:", BUILD_DIR, PROBE_LIB)

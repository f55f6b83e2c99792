"""amdgpu-device-plugin: a Kubernetes device plugin for AMD Instinct MI355X.

The product is a native C++ daemon (``native/``, binary ``amdgpu-device-plugin``)
that discovers GPUs and compute partitions through libamd_smi, serves the kubelet
``v1beta1`` device-plugin gRPC API on Unix sockets, shares GPUs by time-slice
replicas and hands containers ``/dev/kfd`` + ``/dev/dri/renderD*`` on Allocate().

This Python package is the tooling around it -- never a stand-in for it:

* ``utils.native``   -- ctypes binding to ``libadp_capi.so`` (the daemon's own
  allocator / strategy / codec code, for tests and benchmarks);
* ``utils.build``    -- builds the native tree (CMake+Ninja) and the HIP probe;
* ``utils.kubelet``  -- an independent grpcio stub kubelet / plugin client;
* ``utils.harness``  -- launches daemon + stub kubelet in a scratch directory;
* ``models.fixtures``-- MI355X node models (SPX/DPX/QPX/CPX x NPS, 1-8 GPUs,
  xGMI mesh) rendered as amdsmi-mock fixtures;
* ``ops.probe``      -- the HIP visibility/partition probe run on an allocated GPU;
* ``parallel.bench`` -- the multi-rank (torch.distributed) pod-churn benchmark.

Reference parity map: see SURVEY.md section 2 and docs/PARITY.md.
"""

import os

__version__ = "0.1.0"

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD_DIR = os.environ.get("ADP_BUILD_DIR", os.path.join(REPO_ROOT, "build", "native"))
PROBE_DIR = os.path.join(REPO_ROOT, "build", "probe")


def binary(name: str) -> str:
    """Absolute path of a native build artefact (daemon, stub kubelet, libraries)."""
    return os.path.join(BUILD_DIR, name)


DAEMON = binary("amdgpu-device-plugin")
KUBELET_STUB = binary("amdgpu-dp-kubelet")
CAPI_LIB = binary("libadp_capi.so")
MOCK_LIB = binary("libamdsmi_mock.so")
UNIT_TESTS = binary("adp_unit_tests")
PROBE_LIB = os.path.join(PROBE_DIR, "libadp_probe.so")
PROBE_BIN = os.path.join(PROBE_DIR, "amdgpu-dp-probe")

"""Per-device container lists follow KFD topology-node order, not amdsmi order.

Inside a container ROCr makes one agent per KFD topology node whose render node
it can open, in node order, and HIP numbers its devices after the agents. Every
list the plugin hands a container that is indexed by HIP ordinal must follow
that order: HSA_CU_MASK agent numbers, AMD_GPU_MEMORY_LIMIT_MIB / _FRACTION /
_DEVICES and the read-only grant/<ordinal> mounts of the HBM-cap shim. The mock
fixture's "kfd_node" makes KFD order differ from amdsmi's enumeration order,
as it can on a real 8-GPU node.

Reference: the runtime gets an ordered device list from Allocate
(/root/reference/cmd/nvidia-device-plugin/server.go:336-340,397-413); its
container-runtime hook renumbers in that order. There is no hook here, so the
order is the driver's.
"""

import os

import pytest

from k8s_gpu_sharing_plugin_amd import BUILD_DIR, MOCK_LIB
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet, native

SHIM = os.path.join(BUILD_DIR, "libadp_memcap.so")

# GPU 0 (amdsmi order) is KFD node 10, GPU 1 is node 2: HIP device 0 is GPU 1.
A_UUID = "aaaaaaaa-0000-1000-80c0-000000000000"
B_UUID = "bbbbbbbb-0000-1000-80c0-000000000001"


def _swapped(n=2):
    fx = fixtures.node(n)
    fx["gpus"][0]["uuid"] = A_UUID
    fx["gpus"][1]["uuid"] = B_UUID
    fx["gpus"][0]["kfd_node"] = 10
    fx["gpus"][1]["kfd_node"] = 2
    return fx


@pytest.fixture
def served(scratch):
    started = []

    def start(fx, args):
        k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        d = harness.Daemon(scratch, fx, args=args).start()
        started.append((d, k))
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        return d, c, ids
    yield start
    for d, k in started:
        d.stop()
        k.stop()


def test_snapshot_reports_kfd_node_and_hip_id(scratch):
    path = fixtures.write(_swapped(), scratch + ".fx")
    os.environ["AMDSMI_MOCK_FIXTURE"] = path
    snap = native.snapshot(MOCK_LIB)
    assert [g["kfd_node"] for g in snap["gpus"]] == [10, 2]
    assert [g["partitions"][0]["hip_id"] for g in snap["gpus"]] == [1, 0]  # the mock ranks by node
    assert [g["node_index"] for g in snap["gpus"]] == [0, 1]  # index IDs stay amdsmi's


def test_time_slice_spread_pod_masks_follow_kfd_order(served):
    """A 2-GPU time-slice pod under --replica-cu-mask: agent 0 is the GPU with
    the lower KFD node (amdsmi's GPU 1), so its replica's CU range comes first."""
    d, c, ids = served(_swapped(), ["--resource-config", "gpu:sharedgpu:4", "--replica-cu-mask"])
    a = [i for i in ids if i.startswith(A_UUID)]
    b = [i for i in ids if i.startswith(B_UUID)]
    envs = dict(c.allocate([a[0], b[2]]).container_responses[0].envs)
    # GPU A (amdsmi 0, HIP 1) replica 0 -> CUs 0-63; GPU B (amdsmi 1, HIP 0) replica 2 -> 128-191
    assert envs["HSA_CU_MASK"] == "0:128-191;1:0-63"
    assert "KFD topology order differs from amdsmi order" in d.log()
    c.close()


def test_memory_unit_grant_lists_and_mounts_follow_kfd_order(served):
    """An unequal 2-GPU memory-unit grant: the MiB list, the fractions, the
    device list and the read-only grant/<HIP ordinal> files all name HIP device
    0 = amdsmi's GPU 1 first; AMD_VISIBLE_DEVICES (uuid strategy) stays sorted."""
    d, c, ids = served(_swapped(), ["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack",
                                    "--replica-cu-mask", "--auto-replica-unit", "mib", "--enforce-memory-units",
                                    "--memcap-lib", SHIM])
    a = sorted(i for i in ids if i.startswith(A_UUID))
    b = sorted(i for i in ids if i.startswith(B_UUID))
    r = c.allocate(a[:5] + b[:2]).container_responses[0]
    envs = dict(r.envs)
    assert envs["AMD_VISIBLE_DEVICES"] == f"{A_UUID},{B_UUID}"  # sorted by ID (stripReplicas order)
    assert envs["AMD_GPU_MEMORY_DEVICES"] == f"{B_UUID},{A_UUID}"  # HIP order
    assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == "2000,5000"
    grants = [(m.container_path, os.path.basename(m.host_path)) for m in r.mounts
              if m.container_path.startswith("/run/amdgpu-dp/grant/")]
    assert grants == [("/run/amdgpu-dp/grant/0", "2000.mib"), ("/run/amdgpu-dp/grant/1", "5000.mib")]
    assert envs["HSA_CU_MASK"].startswith("0:0-") and ";1:0-" in envs["HSA_CU_MASK"]
    # device specs: both render nodes (their order does not number anything)
    assert sorted(s.container_path for s in r.devices) == ["/dev/dri/renderD128", "/dev/dri/renderD136",
                                                           "/dev/kfd"]
    c.close()


def test_index_strategy_lists_devices_in_kfd_order(served):
    d, c, ids = served(_swapped(4), ["--device-id-strategy", "index"])
    # advertised (ListAndWatch) in KFD order too: GPU 1 (node 2), GPU 0 (node 10), 2, 3
    assert ids[:2] == [B_UUID, A_UUID]
    envs = dict(c.allocate([ids[3], ids[1], ids[0]]).container_responses[0].envs)
    assert envs["AMD_VISIBLE_DEVICES"] == "1,0,3"  # index IDs keep amdsmi numbering, listed in HIP order
    c.close()


def test_unreported_kfd_node_keeps_amdsmi_order_and_warns(served):
    fx = _swapped()
    fx["gpus"][0]["kfd_node"] = None
    d, c, ids = served(fx, ["--resource-config", "gpu:sharedgpu:4", "--replica-cu-mask"])
    a = [i for i in ids if i.startswith(A_UUID)]
    b = [i for i in ids if i.startswith(B_UUID)]
    envs = dict(c.allocate([a[0], b[2]]).container_responses[0].envs)
    assert envs["HSA_CU_MASK"] == "0:0-63;1:128-191"  # amdsmi order
    assert "does not report KFD topology nodes" in d.log()
    c.close()


def test_partitions_follow_their_own_kfd_nodes(served):
    """CPX partitions are KFD nodes of their own: a GPU whose partitions have
    lower nodes than another GPU's come first, partition by partition."""
    fx = fixtures.node(2, "CPX", memory="NPS2")
    fx["gpus"][0]["kfd_node"] = 20
    fx["gpus"][1]["kfd_node"] = 2
    d, c, ids = served(fx, ["--partition-strategy", "single", "--device-id-strategy", "index"])
    assert len(ids) == 16  # advertised in KFD order: GPU 1's 8 partitions, then GPU 0's
    envs = dict(c.allocate([ids[8 + 3], ids[7], ids[0]]).container_responses[0].envs)
    assert envs["AMD_VISIBLE_DEVICES"] == "1:0,1:7,0:3"
    c.close()

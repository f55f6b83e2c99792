"""Reference test vectors, run against the daemon's own C++ code via libadp_capi.

cmd/nvidia-device-plugin/replica_test.go:37-96   Test_prioritizeDevices (15 cases)
cmd/nvidia-device-plugin/replica_test.go:120-122 Test_stripReplicas (3 cases)
"""

import pytest

from k8s_gpu_sharing_plugin_amd.utils import native

MISSING = "device '{}' in mustIncludeDeviceIDs is missing from availableDeviceIDs"
NO_DEVICES = "no devices left to allocate"

# name, available, must_include, size, want ids (None = error), want non_unique, want error
CASES = [
    ("Basic", ["a-replica-0", "a-replica-1", "b-replica-1"], [], 1, ["a-replica-0"], False, None),
    ("Multiple Unique", ["a-replica-0", "a-replica-1", "b-replica-1"], [], 2,
     ["a-replica-0", "b-replica-1"], False, None),
    ("NonuniqueError", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"], [], 3,
     ["a-replica-0", "a-replica-1", "b-replica-1"], True, None),
    ("Must Include Greater Utilized", ["a-replica-0", "a-replica-1", "b-replica-1"], ["b-replica-1"], 1,
     ["b-replica-1"], False, None),
    ("Must Include Least Utilized", ["a-replica-0", "a-replica-1", "b-replica-1"], ["a-replica-1"], 1,
     ["a-replica-1"], False, None),
    ("Must Include Two", ["a-replica-0", "a-replica-1", "b-replica-1"], ["a-replica-1"], 2,
     ["a-replica-1", "b-replica-1"], False, None),
    ("NonuniqueError Must Include", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-2", "b-replica-1"],
     ["a-replica-2"], 3, ["a-replica-0", "a-replica-2", "b-replica-1"], True, None),
    ("Must Include", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1", "c-replica-0"],
     ["a-replica-2"], 3, ["a-replica-2", "b-replica-1", "c-replica-0"], False, None),
    ("Must Include Entire Allocated", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"],
     ["a-replica-2", "b-replica-1", "a-replica-1"], 3, ["a-replica-1", "a-replica-2", "b-replica-1"], True, None),
    ("Deterministic", [f"{c}-replica-1" for c in "abcdefgh"], [], 1, ["a-replica-1"], False, None),
    ("OversizedRequest", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"], [], 5, None, False,
     NO_DEVICES),
    ("Undersized", ["a-replica-0", "a-replica-1", "a-replica-2", "b-replica-1"], [], 0, [], False, None),
    ("NoneAvailable", [], [], 1, None, False, NO_DEVICES),
    ("SubsetSame", ["a-replica-0", "a-replica-1"], ["a-replica-2"], 1, None, False, MISSING.format("a-replica-2")),
    ("SubsetDifferent", ["a-replica-0", "a-replica-1"], ["b-replica-2"], 1, None, False,
     MISSING.format("b-replica-2")),
]


@pytest.mark.parametrize("name,avail,must,size,want,non_unique,err", CASES, ids=[c[0] for c in CASES])
def test_prioritize_devices_reference_vectors(name, avail, must, size, want, non_unique, err):
    if err is not None:
        with pytest.raises(native.NativeError) as e:
            native.prioritize(avail, must, size)
        assert str(e.value) == err
        return
    ids, nu = native.prioritize(avail, must, size)
    assert ids == want
    assert nu == non_unique


@pytest.mark.parametrize("ids,want", [
    (["b-replica-5", "a-replica-1", "a-replica-0"], ["a", "b"]),
    (["b-replica-0", "a-replica-1", "a-replica-2", "c-replica-2"], ["a", "b", "c"]),
    ([], []),
])
def test_strip_replicas_reference_vectors(ids, want):
    assert native.strip_replicas(ids) == want


def test_must_include_larger_than_size_is_an_error_not_a_panic():
    # Reference defect B12: make([]string, len(must), size) panics.
    with pytest.raises(native.NativeError):
        native.prioritize(["a-replica-0", "b-replica-0"], ["a-replica-0", "b-replica-0"], 1)


def test_pack_policy_keeps_memory_units_on_one_gpu():
    # B19: a 20-unit gpu-mem-gb request must come from one GPU.
    avail = [f"g{g}-replica-{i}" for g in range(4) for i in range(30 if g else 10)]
    ids, nu = native.prioritize(avail, [], 20, policy="pack")
    assert len(ids) == 20 and not nu
    assert len({i.split("-replica-")[0] for i in ids}) == 1
    # best fit: a GPU with exactly enough room beats a bigger one
    avail = [f"big-replica-{i}" for i in range(40)] + [f"fit-replica-{i}" for i in range(20)]
    ids, _ = native.prioritize(avail, [], 20, policy="pack")
    assert {i.split("-replica-")[0] for i in ids} == {"fit"}


def test_spread_vs_pack_on_the_same_input():
    avail = [f"{g}-replica-{i}" for g in "ab" for i in range(4)]
    spread, nu = native.prioritize(avail, [], 2)
    assert {i.split("-replica-")[0] for i in spread} == {"a", "b"} and not nu
    pack, _ = native.prioritize(avail, [], 2, policy="pack")
    assert len({i.split("-replica-")[0] for i in pack}) == 1
